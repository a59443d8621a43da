// Host reader of the preprocessor's input: the reference's block / line / sampling semantics
// (lddl/dask/readers.py:60-71 over dask.bag.read_text + random_sample, split_id_text 131-136)
// and the document shuffle of lddl/dask/bert/pretrain.py:100-111 as lddl_amd defines it per
// shuffle group (CPython's Random(seed).shuffle), in C++ threads instead of per-line Python.
//
// Python semantics kept exactly:
//   * every block is decoded strictly (dask decodes whole blocks): malformed UTF-8 anywhere in a
//     block is an error, sampled out or not (Python's decoder rules: no overlongs, surrogates or
//     code points > U+10FFFF);
//   * lines = block.split('\n'), each str.strip()ed (str.isspace code points at both ends), empty
//     ones dropped, then kept iff random() < ratio from the block's MT state (dask 2021.10
//     random_state_data_python: 624 words + index);
//   * shuffle: random.Random(seed).shuffle (seed(int) = init_by_array over the 32-bit limbs of
//     abs(seed); for i = n-1 .. 1: j = _randbelow(i + 1) by getrandbits rejection);
//   * a document's text is what follows the first str.isspace code point of its line.
#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <fcntl.h>
#include <unistd.h>

#include "common.h"
#include "lddl_amd.h"

namespace lddl {
namespace {

// ---- CPython MT19937 (Modules/_randommodule.c) ----------------------------------------------
struct PyMT {
  uint32_t mt[624];
  int idx = 624;

  void twist() {
    for (int i = 0; i < 624; ++i) {
      const uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % 624] & 0x7fffffffu);
      mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    idx = 0;
  }
  uint32_t u32() {
    if (idx >= 624) twist();
    uint32_t y = mt[idx++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }
  double random() {  // genrand_res53
    const uint32_t a = u32() >> 5, b = u32() >> 6;
    return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
  }
  uint32_t randbelow(uint32_t n) {  // _randbelow_with_getrandbits, n >= 1
    int k = 0;
    while (k < 32 && (n >> k)) ++k;
    uint32_t r = u32() >> (32 - k);
    while (r >= n) r = u32() >> (32 - k);
    return r;
  }
  void seed_u64(uint64_t a) {  // random.seed(a) for a = abs(int) < 2^64: init_by_array
    const uint32_t key[2] = {(uint32_t)a, (uint32_t)(a >> 32)};
    const int klen = key[1] ? 2 : 1;
    mt[0] = 19650218u;
    for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    int i = 1, j = 0;
    for (int k = 624; k; --k) {
      mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
      ++i;
      ++j;
      if (i >= 624) { mt[0] = mt[623]; i = 1; }
      if (j >= klen) j = 0;
    }
    for (int k = 623; k; --k) {
      mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
      ++i;
      if (i >= 624) { mt[0] = mt[623]; i = 1; }
    }
    mt[0] = 0x80000000u;
    idx = 624;
  }
};

// ---- UTF-8 ----------------------------------------------------------------------------------
// offset of the first byte of b[0, n) that does not begin or continue a well-formed sequence, or
// -1 (CPython's strict decoder)
int64_t utf8_first_bad(const uint8_t* b, int64_t n) {
  int64_t i = 0;
  while (i < n) {
    // ASCII runs 8 bytes at a time
    while (i + 8 <= n) {
      uint64_t w;
      memcpy(&w, b + i, 8);
      if (w & 0x8080808080808080ull) break;
      i += 8;
    }
    if (i >= n) break;
    const uint8_t c = b[i];
    if (c < 0x80) { ++i; continue; }
    int len;
    uint8_t lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) len = 2;
    else if (c >= 0xE0 && c <= 0xEF) {
      len = 3;
      if (c == 0xE0) lo = 0xA0;
      if (c == 0xED) hi = 0x9F;
    } else if (c >= 0xF0 && c <= 0xF4) {
      len = 4;
      if (c == 0xF0) lo = 0x90;
      if (c == 0xF4) hi = 0x8F;
    } else {
      return i;
    }
    if (i + 1 >= n || b[i + 1] < lo || b[i + 1] > hi) return i;
    for (int k = 2; k < len; ++k)
      if (i + k >= n || (b[i + k] & 0xC0) != 0x80) return i;
    i += len;
  }
  return -1;
}

// str.isspace() (Python 3.10)
inline bool py_space(uint32_t cp) {
  if (cp < 0x80) return (cp >= 0x09 && cp <= 0x0D) || (cp >= 0x1C && cp <= 0x20);
  return cp == 0x85 || cp == 0xA0 || cp == 0x1680 || (cp >= 0x2000 && cp <= 0x200A) ||
         cp == 0x2028 || cp == 0x2029 || cp == 0x202F || cp == 0x205F || cp == 0x3000;
}

// code point at b[i] of valid UTF-8, its length in *len
inline uint32_t cp_at(const uint8_t* b, int64_t i, int* len) {
  const uint32_t c = b[i];
  if (c < 0x80) { *len = 1; return c; }
  if (c < 0xE0) { *len = 2; return ((c & 0x1F) << 6) | (b[i + 1] & 0x3F); }
  if (c < 0xF0) {
    *len = 3;
    return ((c & 0x0F) << 12) | ((b[i + 1] & 0x3F) << 6) | (b[i + 2] & 0x3F);
  }
  *len = 4;
  return ((c & 0x07) << 18) | ((b[i + 1] & 0x3F) << 12) | ((b[i + 2] & 0x3F) << 6) |
         (b[i + 3] & 0x3F);
}

// str.strip() of valid UTF-8 [a, z): the stripped range
inline void py_strip(const uint8_t* b, int64_t& a, int64_t& z) {
  while (a < z) {
    int l;
    if (!py_space(cp_at(b, a, &l))) break;
    a += l;
  }
  while (z > a) {
    int64_t s = z - 1;
    while (s > a && (b[s] & 0xC0) == 0x80) --s;
    int l;
    if (!py_space(cp_at(b, s, &l))) break;
    z = s;
  }
}

struct Line {
  int64_t off, len;  // inside the block buffer
};

struct BlockData {
  std::vector<uint8_t> buf;
  std::vector<Line> lines;  // kept (stripped, non-empty, sampled) lines
  int64_t bad = -1;         // first malformed byte (block-relative), -1 = valid
  std::string err;
};

}  // namespace
}  // namespace lddl

struct lddl_reader {
  std::vector<lddl::BlockData> blocks;
  std::vector<std::pair<int32_t, int32_t>> docs;  // output order: (block, line) of each document
  std::vector<int64_t> block_ndocs;
  std::vector<int64_t> tstart, tlen;  // text after the id, per document (block-buffer relative)
  int n_threads = 1;
};

using namespace lddl;

namespace {

void read_one(lddl_reader* R, int64_t i, const char* path, int64_t start, int64_t end,
              const uint32_t* st, double ratio) {
  BlockData& B = R->blocks[i];
  const int64_t n = end > start ? end - start : 0;
  B.buf.resize((size_t)n);
  if (n) {
    const int fd = open(path, O_RDONLY);
    if (fd < 0) {
      B.err = std::string("cannot open ") + path + ": " + strerror(errno);
      return;
    }
    int64_t got = 0;
    while (got < n) {
      const ssize_t r = pread(fd, B.buf.data() + got, (size_t)(n - got), (off_t)(start + got));
      if (r <= 0) {
        B.err = std::string("short read of ") + path;
        close(fd);
        return;
      }
      got += r;
    }
    close(fd);
  }
  const uint8_t* b = B.buf.data();
  B.bad = utf8_first_bad(b, n);
  if (B.bad >= 0) return;
  PyMT mt;
  if (st) {
    memcpy(mt.mt, st, sizeof(mt.mt));
    mt.idx = (int)st[624];
  }
  int64_t a = 0;
  while (a <= n) {
    const uint8_t* nl = a < n ? static_cast<const uint8_t*>(memchr(b + a, '\n', (size_t)(n - a)))
                              : nullptr;
    const int64_t e = nl ? nl - b : n;
    int64_t s = a, z = e;
    py_strip(b, s, z);
    if (z > s && (!st || mt.random() < ratio)) B.lines.push_back(Line{s, z - s});
    a = e + 1;
  }
}

template <typename F>
void parallel_for(int64_t n, int threads, F f) {
  threads = (int)std::max<int64_t>(1, std::min<int64_t>(threads, n));
  std::atomic<int64_t> next(0);
  auto work = [&]() {
    for (int64_t i; (i = next.fetch_add(1)) < n;) f(i);
  };
  std::vector<std::thread> th;
  for (int t = 1; t < threads; ++t) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
}

}  // namespace

extern "C" int lddl_read_groups(int64_t n_blocks, const char* const* paths, const int64_t* starts,
                                const int64_t* ends, const uint32_t* mt_states, double ratio,
                                int64_t n_groups, const int64_t* group_off,
                                const uint64_t* group_seed_abs, int n_threads, lddl_reader** out,
                                int64_t* n_docs, int64_t* n_text, int64_t* bad) {
  if (!out || n_blocks < 0 || n_groups < 0 || (n_groups && group_off[n_groups] != n_blocks))
    LDDL_FAIL(-1, "lddl_read_groups: bad arguments");
  *out = nullptr;
  lddl_reader* R = new lddl_reader;
  R->n_threads = std::max(1, n_threads);
  R->blocks.resize((size_t)n_blocks);
  parallel_for(n_blocks, R->n_threads, [&](int64_t i) {
    read_one(R, i, paths[i], starts[i], ends[i], mt_states ? mt_states + 625 * i : nullptr, ratio);
  });
  for (int64_t i = 0; i < n_blocks; ++i) {
    if (!R->blocks[i].err.empty()) {
      const std::string e = R->blocks[i].err;
      delete R;
      LDDL_FAIL(-1, "%s", e.c_str());
    }
    if (R->blocks[i].bad >= 0) {
      if (bad) {
        bad[0] = i;
        bad[1] = R->blocks[i].bad;
      }
      delete R;
      LDDL_FAIL(-2, "invalid UTF-8 in block %lld at byte %lld", (long long)i,
                (long long)(starts[i] + (bad ? bad[1] : 0)));
    }
  }
  // each group's documents shuffled over its blocks (pretrain.py:100-111, per shuffle group)
  R->block_ndocs.assign((size_t)n_blocks, 0);
  std::vector<int64_t> doc_base((size_t)n_groups + 1, 0);
  for (int64_t g = 0; g < n_groups; ++g) {
    int64_t c = 0;
    for (int64_t i = group_off[g]; i < group_off[g + 1]; ++i) {
      R->block_ndocs[i] = (int64_t)R->blocks[i].lines.size();
      c += R->block_ndocs[i];
    }
    doc_base[g + 1] = doc_base[g] + c;
  }
  const int64_t total = doc_base[n_groups];
  R->docs.resize((size_t)total);
  parallel_for(n_groups, R->n_threads, [&](int64_t g) {
    std::pair<int32_t, int32_t>* d = R->docs.data() + doc_base[g];
    int64_t k = 0;
    for (int64_t i = group_off[g]; i < group_off[g + 1]; ++i)
      for (int32_t l = 0; l < (int32_t)R->blocks[i].lines.size(); ++l) d[k++] = {(int32_t)i, l};
    PyMT mt;
    mt.seed_u64(group_seed_abs[g]);
    for (int64_t i = k - 1; i >= 1; --i) std::swap(d[i], d[mt.randbelow((uint32_t)(i + 1))]);
  });
  // split_id_text: the text after the line's first whitespace code point
  R->tstart.resize((size_t)total);
  R->tlen.resize((size_t)total);
  parallel_for((total + 4095) / 4096, R->n_threads, [&](int64_t c) {
    for (int64_t q = c * 4096; q < std::min(total, (c + 1) * 4096); ++q) {
      const BlockData& B = R->blocks[R->docs[q].first];
      const Line& L = B.lines[R->docs[q].second];
      const uint8_t* b = B.buf.data();
      int64_t i = L.off, e = L.off + L.len;
      int l = 0;
      while (i < e) {
        if (py_space(cp_at(b, i, &l))) break;
        i += l;
      }
      if (i < e) i += l;
      R->tstart[q] = i;
      R->tlen[q] = e - i;
    }
  });
  int64_t nt = 0;
  for (int64_t q = 0; q < total; ++q) nt += R->tlen[q];
  *out = R;
  if (n_docs) *n_docs = total;
  if (n_text) *n_text = nt;
  return 0;
}

extern "C" int lddl_read_fill(lddl_reader* R, uint8_t* text, int64_t* doc_off,
                              int64_t* block_ndocs) {
  if (!R) LDDL_FAIL(-1, "null reader");
  const int64_t total = (int64_t)R->docs.size();
  doc_off[0] = 0;
  for (int64_t q = 0; q < total; ++q) doc_off[q + 1] = doc_off[q] + R->tlen[q];
  parallel_for((total + 1023) / 1024, R->n_threads, [&](int64_t c) {
    for (int64_t q = c * 1024; q < std::min(total, (c + 1) * 1024); ++q)
      if (R->tlen[q])
        memcpy(text + doc_off[q], R->blocks[R->docs[q].first].buf.data() + R->tstart[q],
               (size_t)R->tlen[q]);
  });
  if (block_ndocs)
    memcpy(block_ndocs, R->block_ndocs.data(), sizeof(int64_t) * R->block_ndocs.size());
  return 0;
}

extern "C" int lddl_read_counts(const lddl_reader* R, int64_t* block_ndocs, int64_t* doc_len) {
  if (!R) LDDL_FAIL(-1, "null reader");
  if (block_ndocs)
    memcpy(block_ndocs, R->block_ndocs.data(), sizeof(int64_t) * R->block_ndocs.size());
  if (doc_len) memcpy(doc_len, R->tlen.data(), sizeof(int64_t) * R->tlen.size());
  return 0;
}

extern "C" int lddl_read_fill_range(lddl_reader* R, int64_t d0, int64_t d1, uint8_t* text,
                                    int64_t* doc_off) {
  if (!R || d0 < 0 || d1 < d0 || d1 > (int64_t)R->docs.size()) LDDL_FAIL(-1, "bad doc range");
  const int64_t n = d1 - d0;
  doc_off[0] = 0;
  for (int64_t q = 0; q < n; ++q) doc_off[q + 1] = doc_off[q] + R->tlen[d0 + q];
  parallel_for((n + 1023) / 1024, R->n_threads, [&](int64_t c) {
    for (int64_t q = c * 1024; q < std::min(n, (c + 1) * 1024); ++q) {
      const int64_t d = d0 + q;
      if (R->tlen[d])
        memcpy(text + doc_off[q], R->blocks[R->docs[d].first].buf.data() + R->tstart[d],
               (size_t)R->tlen[d]);
    }
  });
  return 0;
}

// dask 2021.10 random_state_data_python(n, seed): n states of 624 words, each word
// Random(seed).randint(0, 2**32) drawn in order (randint -> _randbelow(2**32 + 1) ->
// getrandbits(33): two words, the second's top bit as bit 32, redrawn while >= 2**32 + 1).
// out[625 * i + 624] = 624 (the state's index).
extern "C" int lddl_random_state_data(int64_t n, uint64_t seed_abs, uint32_t* out) {
  if (n < 0 || !out) LDDL_FAIL(-1, "bad arguments");
  PyMT mt;
  mt.seed_u64(seed_abs);
  for (int64_t i = 0; i < n; ++i) {
    for (int k = 0; k < 624; ++k) {
      uint64_t v;
      do {
        const uint64_t lo = mt.u32();
        const uint64_t hi = mt.u32() >> 31;
        v = lo | (hi << 32);
      } while (v > (1ull << 32));
      // randint(0, 2**32) may be 2**32 itself: CPython's setstate() stores each word as
      // (uint32_t)PyLong_AsUnsignedLong(w), i.e. 0
      out[625 * i + k] = (uint32_t)v;
    }
    out[625 * i + 624] = 624;
  }
  return 0;
}

extern "C" int lddl_read_free(lddl_reader* R) {
  delete R;
  return 0;
}
