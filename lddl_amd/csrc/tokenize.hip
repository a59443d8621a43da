// Sentence -> WordPiece ids on the GPU.
//
// Replaces the per-sentence `tokenizer.tokenize(s, max_length=512, truncation=True)` call of
// lddl/dask/bert/pretrain.py:79-80 (HF BertTokenizerFast: added-token split on raw text,
// BertNormalizer, BertPreTokenizer, WordPiece; see oracle/lddl_oracle.c for the restated
// algorithm and tools/make_norm_tables.py for the per-code-point table).
//
// Output layout (no prefix sum needed): every code point normalises to at most as many chars
// as its UTF-8 bytes and every piece consumes >= 1 char, so a sentence never has more pieces than
// bytes; sentence s writes its pieces to ids[sent_off[s] ...] and its kept count (<= max_pieces)
// to sent_len[s] (bit 30 set if the kept pieces contain a literal [CLS]/[SEP]).
//
// Kernels:
//   tokenize_batch_kernel  the product path. Persistent workgroups of kBW waves (one per CU,
//                          sharing an LDS Bloom filter of the vocab); each wave streams its
//                          sentences (dynamic chunks) in 64-byte windows, one byte per lane. Lanes
//                          classify code points, ballots find the pre-tokenizer units, which go
//                          to an LDS queue spanning sentences; every kSF queued units are
//                          resolved in two phases (A: one vocab probe per unit, B: greedy
//                          longest-match WordPiece of the multi-piece / non-ASCII units only)
//                          and placed in queue order by a segmented scan (details above the
//                          kernel). A unit that does not fit (> kNorm normalised bytes, > kPcs
//                          pieces) sends its sentence to the fallback list.
//   tokenize_lane_kernel   one lane per listed sentence, sequential (unbounded words, 100-char
//                          rule); also the whole-corpus path when LDDL_TOKENIZE_PATH=lane.
//   tokenize_wave_kernel   round-1 design, one wavefront per sentence with no cross-sentence
//                          queue; kept only as the LDDL_TOKENIZE_PATH=wave diagnostic.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>
#include <cstdio>

#include "common.h"
#include "ctx.h"
#include "device.h"
#include "lddl_amd.h"

namespace lddl {
namespace {

constexpr int kBlock = 128;       // threads per workgroup
constexpr int kWordStride = 420;  // bytes per lane word buffer: 100 chars * 4 B + pad; 105
                                  // dwords (odd) so lanes hit distinct LDS banks

__device__ inline uint32_t tab_entry(const Tables& T, uint32_t cp) {
  if (cp > 0x10FFFF) return kDrop << 30;
  return T.pages[(uint32_t)T.l1[cp >> 8] * 256u + (cp & 255u)];
}

__device__ inline uint32_t utf8_next(const uint8_t* b, int64_t end, int64_t& i) {
  const uint32_t c = b[i];
  if (c < 0x80) { ++i; return c; }
  const int len = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : c >= 0xC0 ? 2 : 1;
  if (len == 1 || i + len > end) { ++i; return 0xFFFD; }
  uint32_t cp = c & (0x7Fu >> len);
  for (int k = 1; k < len; ++k) {
    const uint32_t d = b[i + k];
    if ((d & 0xC0) != 0x80) { ++i; return 0xFFFD; }
    cp = (cp << 6) | (d & 0x3F);
  }
  i += len;
  return cp;
}

__device__ inline int put_utf8(uint8_t* o, uint32_t cp) {
  if (cp < 0x80) { o[0] = (uint8_t)cp; return 1; }
  if (cp < 0x800) { o[0] = 0xC0 | (cp >> 6); o[1] = 0x80 | (cp & 63); return 2; }
  if (cp < 0x10000) {
    o[0] = 0xE0 | (cp >> 12); o[1] = 0x80 | ((cp >> 6) & 63); o[2] = 0x80 | (cp & 63);
    return 3;
  }
  o[0] = 0xF0 | (cp >> 18); o[1] = 0x80 | ((cp >> 12) & 63); o[2] = 0x80 | ((cp >> 6) & 63);
  o[3] = 0x80 | (cp & 63);
  return 4;
}

// Vocab lookup of w[s, s+len) with or without the "##" continuation prefix.
__device__ int32_t lookup(const Tables& T, const uint8_t* w, int s, int len, uint32_t cont) {
  uint64_t k0 = 0;
  uint32_t k1 = 0;
  const int n0 = len < 8 ? len : 8;
  for (int i = 0; i < n0; ++i) k0 |= (uint64_t)w[s + i] << (8 * i);
  for (int i = 8; i < len && i < 12; ++i) k1 |= (uint32_t)w[s + i] << (8 * (i - 8));
  const uint32_t want = kMetaValid | (cont ? kMetaCont : 0u) | (len > 12 ? kMetaLong : 0u) |
                        ((uint32_t)len << 21);
  for (uint32_t slot = (uint32_t)vhash(k0, k1, len, cont) & T.vmask;; slot = (slot + 1) & T.vmask) {
    const VEnt e = T.vhash[slot];
    if (!(e.meta & kMetaValid)) return -1;
    if (e.k0 == k0 && e.k1 == k1 && (e.meta & ~0x1FFFFFu) == want) {
      const int32_t id = meta_id(e.meta);
      if (len <= 12) return id;
      const uint8_t* p = T.vbytes + T.voff[id];
      bool ok = true;
      for (int i = 12; i < len; ++i) ok &= p[i] == w[s + i];
      if (ok) return id;
    }
  }
}

struct Sink {
  int32_t* out;  // sentence region ids[sent_off[s] ...]
  int32_t n;     // pieces emitted so far (may run past max_pieces inside the region)
};

// Greedy longest-match WordPiece of one normalised word (HF tokenizers WordPiece::tokenize).
__device__ void wordpiece(const Tables& T, const uint8_t* w, int nb, int nc, bool overflow,
                          Sink& sk) {
  if (nc == 0) return;
  if (overflow || nc > 100) { sk.out[sk.n++] = T.special_id[kUnk]; return; }
  const int first = sk.n;
  int start = 0;
  while (start < nb) {
    int end = nb < start + T.max_piece_bytes ? nb : start + T.max_piece_bytes;
    int32_t found = -1;
    for (; end > start; --end) {
      if (end < nb && (w[end] & 0xC0) == 0x80) continue;  // not a char boundary
      found = lookup(T, w, start, end - start, start > 0);
      if (found >= 0) break;
    }
    if (found < 0) {
      sk.n = first;
      sk.out[sk.n++] = T.special_id[kUnk];
      return;
    }
    sk.out[sk.n++] = found;
    start = end;
  }
}

__device__ inline bool match_special(const uint8_t* b, int64_t i, int64_t end, int k) {
  // "[PAD]" "[UNK]" "[CLS]" "[SEP]" "[MASK]"
  const char* s = k == 0 ? "[PAD]" : k == 1 ? "[UNK]" : k == 2 ? "[CLS]" : k == 3 ? "[SEP]" : "[MASK]";
  const int L = k == 4 ? 6 : 5;
  if (i + L > end) return false;
  for (int j = 1; j < L; ++j)
    if (b[i + j] != (uint8_t)s[j]) return false;
  return true;
}

__global__ void __launch_bounds__(kBlock) tokenize_lane_kernel(
    Tables T, const uint8_t* __restrict__ text, const int64_t* __restrict__ sent_off,
    int64_t n_sent, int32_t max_pieces, int32_t* __restrict__ ids, int32_t* __restrict__ sent_len,
    const int32_t* __restrict__ list, const uint32_t* __restrict__ list_n) {
  __shared__ uint8_t wbuf_all[kBlock * kWordStride];
  const int64_t n_items = list ? (int64_t)*list_n : n_sent;
  for (int64_t it = (int64_t)blockIdx.x * kBlock + threadIdx.x; it < n_items;
       it += (int64_t)gridDim.x * kBlock) {
  const int64_t s = list ? (int64_t)list[it] : it;
  uint8_t* w = wbuf_all + threadIdx.x * kWordStride;
  const int64_t b0 = sent_off[s], b1 = sent_off[s + 1];
  Sink sk{ids + b0, 0};
  int32_t flags = 0;
  int nb = 0, nc = 0;
  bool ovf = false;
  int64_t i = b0;
  while (i < b1 && sk.n < max_pieces) {
    if (text[i] == '[') {
      int best = -1;
      for (int k = 0; k < kNumSpecial; ++k)
        if (T.special_id[k] >= 0 && match_special(text, i, b1, k)) { best = k; break; }
      if (best >= 0) {
        wordpiece(T, w, nb, nc, ovf, sk);
        nb = nc = 0;
        ovf = false;
        if (sk.n < max_pieces && (best == kCls || best == kSep)) flags = kLenHasClsSep;
        sk.out[sk.n++] = T.special_id[best];
        i += best == kMask ? 6 : 5;
        continue;
      }
    }
    const uint32_t cp = utf8_next(text, b1, i);
    const uint32_t e = tab_entry(T, cp);
    const uint32_t cls = e >> 30;
    if (cls == kDrop) continue;
    if (cls == kSpace) {
      wordpiece(T, w, nb, nc, ovf, sk);
      nb = nc = 0;
      ovf = false;
      continue;
    }
    uint8_t ob[12];
    int olen, ochars = 1;
    if (e & kIdent) olen = put_utf8(ob, cp);
    else if (e & kMulti) {
      const uint8_t* p = T.pool + (e & 0xFFFFFFu);
      olen = p[0];
      ochars = p[1];
      for (int k = 0; k < olen; ++k) ob[k] = p[2 + k];
    } else olen = put_utf8(ob, e & 0x1FFFFFu);
    if (cls == kIso) {
      wordpiece(T, w, nb, nc, ovf, sk);
      for (int k = 0; k < olen; ++k) w[k] = ob[k];
      wordpiece(T, w, olen, 1, false, sk);
      nb = nc = 0;
      ovf = false;
      continue;
    }
    if (ovf || nc + ochars > 100) { ovf = true; nc += ochars; continue; }
    for (int k = 0; k < olen; ++k) w[nb + k] = ob[k];
    nb += olen;
    nc += ochars;
  }
  if (sk.n < max_pieces) wordpiece(T, w, nb, nc, ovf, sk);
  sent_len[s] = (sk.n < max_pieces ? sk.n : max_pieces) | flags;
  }
}

// ---------------------------------------------------------------------------------------------
// Wave tokenizer
// ---------------------------------------------------------------------------------------------
constexpr int kTW = 4;     // waves per workgroup
constexpr int kPcs = 8;    // pieces per unit held per lane (more -> fallback)
constexpr int kNorm = 32;  // normalised bytes per unit on the generic path (more -> fallback)

// unit categories per byte position
enum : uint32_t { kCatRun = 0, kCatSep = 1, kCatIso = 2, kCatSpecial = 3 };

struct alignas(16) WaveLds {
  uint8_t us[64], ue[64], uk[64];  // unit k: first byte, last byte (window-relative), kind
  int32_t pcs[kPcs * 64];          // lane l's pieces at pcs[64 q + l]
  alignas(16) uint8_t nrm[64 * kNorm];  // lane l's normalised word (generic path)
};

// Order this wave's LDS writes before its later LDS reads of other lanes' data (the waves of a
// workgroup work on different sentences, so a workgroup barrier would not be uniform).
__device__ inline uint64_t lanes_below() { return (1ull << lane_id()) - 1ull; }

__device__ inline int match_special_at(const Tables& T, const uint8_t* b, int64_t i, int64_t end) {
  for (int k = 0; k < kNumSpecial; ++k)
    if (T.special_id[k] >= 0 && match_special(b, i, end, k)) return k;
  return -1;
}

// Up to 32 bytes of a word as four little-endian 64-bit words (bytes past the word: don't care,
// every use masks by length).
struct B32 {
  uint64_t w0, w1, w2, w3;
};

// bytes [s, 32) moved to the front (s in 0..31)
__device__ inline B32 shr_bytes(const B32& v, int s) {
  const int q = s >> 3, r = (s & 7) * 8;
  uint64_t a0 = q == 0 ? v.w0 : q == 1 ? v.w1 : q == 2 ? v.w2 : v.w3;
  uint64_t a1 = q == 0 ? v.w1 : q == 1 ? v.w2 : q == 2 ? v.w3 : 0ull;
  uint64_t a2 = q == 0 ? v.w2 : q == 1 ? v.w3 : 0ull;
  uint64_t a3 = q == 0 ? v.w3 : 0ull;
  if (r) {
    a0 = (a0 >> r) | (a1 << (64 - r));
    a1 = (a1 >> r) | (a2 << (64 - r));
    a2 = (a2 >> r) | (a3 << (64 - r));
    a3 >>= r;
  }
  return B32{a0, a1, a2, a3};
}

// The pieces of one unit: the lane's column of an LDS buffer (lane l's piece q at b[64 q]).
struct Pcs {
  int32_t* b;
  __device__ void put(int n, int32_t v) { b[64 * n] = v; }
  __device__ int32_t get(int q) const { return b[64 * q]; }
};

// Diagnostic build: work counters of phase B (per lane; summed at the kernel's end).
struct TokStats {
#ifdef LDDL_STAMPS
  uint64_t c[10];
  __device__ void add(int i, uint64_t v) { c[i] += v; }
  // once per wave-level iteration: only the first active lane counts
  __device__ void wave(int i) {
    const uint64_t m = __builtin_amdgcn_ballot_w64(true);
    if ((uint32_t)__lane_id() == (uint32_t)__builtin_ctzll(m)) c[i] += 1;
  }
#else
  __device__ void add(int, uint64_t) {}
  __device__ void wave(int) {}
#endif
};

// Bytes 8 .. len-1 (len 13..32) of a against piece id's zero-padded 32-byte copy (the hash key
// already matched bytes 0..11).
__device__ inline bool tail_match(const Tables& T, int32_t id, const B32& a, int len) {
  const ulonglong2* p = reinterpret_cast<const ulonglong2*>(T.vlong + 4 * (int64_t)id);
  const ulonglong2 lo = p[0], hi = p[1];
  const uint64_t d = keep_bytes(lo.y ^ a.w1, len - 8) | keep_bytes(hi.x ^ a.w2, len - 16) |
                     keep_bytes(hi.y ^ a.w3, len - 24);
  return d == 0;
}

// Vocab probe of the first `len` (1..32) bytes of a: exact key for <= 12 bytes (k0 = bytes 0..7,
// k1 = bytes 8..11), longer pieces confirmed against their 32-byte copies.

// probe32 split in two, so that several probes' first table loads are in flight together:
// probe_first computes the key and issues the load of the home slot, probe_finish examines it
// and walks the collision chain (rarely more than the home slot).
struct Probe {
  uint64_t k0;
  uint32_t k1, want, slot;
  VEnt e;
};
__device__ inline Probe probe_first(const Tables& T, const B32& a, int len, uint32_t cont) {
  Probe q;
  q.k0 = keep_bytes(a.w0, len);
  q.k1 = (uint32_t)keep_bytes(a.w1, len - 8 < 4 ? len - 8 : 4);
  q.want = kMetaValid | (cont ? kMetaCont : 0u) | (len > 12 ? kMetaLong : 0u) | ((uint32_t)len << 21);
  q.slot = (uint32_t)vhash(q.k0, q.k1, len, cont) & T.vmask;
  q.e = T.vhash[q.slot];
  return q;
}
__device__ inline int32_t probe_finish(const Tables& T, const B32& a, int len, Probe q) {
  for (;;) {
    if (!(q.e.meta & kMetaValid)) return -1;
    if (q.e.k0 == q.k0 && q.e.k1 == q.k1 && (q.e.meta & ~0x1FFFFFu) == q.want &&
        (len <= 12 || tail_match(T, meta_id(q.e.meta), a, len)))
      return meta_id(q.e.meta);
    q.slot = (q.slot + 1) & T.vmask;
    q.e = T.vhash[q.slot];
  }
}

// Bloom candidates for the pieces starting at a's first byte: bit L-1 set iff the filter may
// contain (cont, bytes[0, L)), L = 1 .. maxl (<= 32). (Round 5 read the filter words of 2 / 4 / 8
// lengths before testing any: 19.31 / 21.1 / 22.9 ms per 2 GB against 19.32, the grouped reads
// cost registers; profiles/r05i_tok_variants.txt, code on branch ab/tok-cp-variants.)
__device__ inline uint32_t bloom_candidates32(const uint32_t* bloom, const B32& a, int maxl,
                                              uint32_t cont, TokStats* ts = nullptr) {
  uint32_t h = 0, cand = 0;
#pragma unroll
  for (int L = 1; L <= 32; ++L) {
    // wave-uniform exit (lanes past their own maxl compute don't-care bits, masked below): no
    // exec-mask bookkeeping per length
    if (!ballot(L <= maxl)) break;
    if (ts) {
      ts->wave(4);
      ts->add(5, L <= maxl);
    }
    const uint64_t wv = L <= 8 ? a.w0 : L <= 16 ? a.w1 : L <= 24 ? a.w2 : a.w3;
    const uint32_t byte = (uint32_t)(wv >> (8 * ((L - 1) & 7))) & 0xFFu;
    h = h * kBloomP + byte + 1u;
    const uint32_t x = bloom_mix(h, (uint32_t)L, cont);
    const uint32_t msk = bloom_bits(x);
    cand |= (bloom[bloom_word(x)] & msk) == msk ? 1u << (L - 1) : 0u;
  }
  return maxl >= 32 ? cand : cand & ((1u << maxl) - 1u);
}

// One greedy longest-match step of a word held in registers: the longest vocab piece (continuation
// iff start > 0) starting at byte `start`; returns its id and length, or -1 (no piece matches:
// the word is [UNK]). Per step, the Bloom filter (LDS) gives the lengths that may be pieces (every
// vocab piece is in it: the longest candidate that hits is the greedy match), and the two longest
// candidates' home slots are loaded together, so a lane waits on ONE table round trip per piece
// in the common case. first_probe_missed: phase A already probed the whole word (start 0).
__device__ inline int32_t piece_step(const Tables& T, const uint32_t* bloom, const B32& v, int nb,
                                     uint64_t ends, int start, bool first_probe_missed, int& out_len,
                                     TokStats* ts = nullptr) {
  const B32 a = shr_bytes(v, start);
  const uint32_t cont = start > 0;
  const uint64_t e = ends >> start;  // bit L: a piece of length L may end here
  int len = nb - start < T.max_piece_bytes ? nb - start : T.max_piece_bytes;
  {  // the longest length <= len that ends on a character boundary (bit L-1 of okl: length L)
    const uint64_t okl = (e >> 1) & ((1ull << len) - 1ull);
    len = okl ? 64 - __clzll(okl) : 0;
  }
  uint32_t cand = len > 0 ? bloom_candidates32(bloom, a, len, cont, ts) & (uint32_t)(e >> 1) : 0u;
  // (the caller may already know that the whole word is not one piece)
  if (first_probe_missed && start == 0 && len == nb) cand &= ~(1u << (len - 1));
  int32_t id = -1;
  while (cand) {
    if (ts) {
      ts->wave(6);
      ts->add(7, 1);
    }
    const int l1 = 32 - __clz(cand);
    const uint32_t r1 = cand & ~(1u << (l1 - 1));
    const int l2 = r1 ? 32 - __clz(r1) : 0;
    const Probe q1 = probe_first(T, a, l1, cont);
    const Probe q2 = probe_first(T, a, l2 ? l2 : l1, cont);
    id = probe_finish(T, a, l1, q1);
    if (id >= 0) {
      len = l1;
      break;
    }
    if (l2) {
      id = probe_finish(T, a, l2, q2);
      if (id >= 0) {
        len = l2;
        break;
      }
    }
    cand = l2 ? r1 & ~(1u << (l2 - 1)) : 0u;
  }
  out_len = len;
  return id;
}

// Greedy longest-match WordPiece (HF WordPiece::tokenize) of a normalised word of nb <= 32 bytes
// held in registers. ends: bit e set iff a piece may end at byte e (a UTF-8 character boundary;
// all bits for ASCII). Returns the piece count written to pc, or -1 if more than kPcs pieces.
// (Round 3 probed the full length alone first, then two candidates per round trip: 21.9 ms per
// 2 GiB against 20.7 now; three candidates per trip spilled VGPRs and took 22.1 ms, r04o.)
__device__ int wordpiece32(const Tables& T, const uint32_t* bloom, const B32& v, int nb,
                           uint64_t ends, Pcs& pc, bool first_probe_missed = false,
                           TokStats* ts = nullptr) {
  int n = 0, start = 0;
  while (start < nb) {
    if (ts) {
      ts->wave(2);
      ts->add(3, 1);
    }
    int len;
    const int32_t id = piece_step(T, bloom, v, nb, ends, start, first_probe_missed, len, ts);
    if (id < 0) {  // no piece: the whole word is [UNK]
      pc.put(0, T.special_id[kUnk]);
      return 1;
    }
    if (n == kPcs) return -1;
    pc.put(n++, id);
    start += len;
  }
  return n;
}

// Classification of one 64-byte window [pos, pos+64) of a sentence ending at b1 (one byte per
// lane). Returns, in registers, the window's complete units as masks (US: first bytes, UE: last
// bytes; unit k = the k-th bit of each), each start lane's unit kind (0 word run, 1 isolated
// char, 2 + k literal special token k), the start of the next window and the mask of lanes
// holding a byte the register fast path cannot take. The caller stores what it needs.
struct WinResult {
  int n_units;
  int next_lane;  // the next window starts at this lane's byte (64: after lane 63; -1: the last
                  // segment is consumed to its end)
  int64_t next;   // classify_window only: the same as a byte offset
  uint64_t slow;
  uint64_t US, UE;  // unit starts (a trailing incomplete unit included) / complete unit ends
  int ukind;        // this lane's unit kind when its US bit is set
  bool unit_byte;   // this lane's byte belongs to a unit (not a separator)
  bool fallback;    // a unit of >= 64 bytes: the sentence goes to the lane kernel
};

// Per-lane form: this lane's byte offset i, the end b1 of its sentence, and byte = text[i] (any
// value when i >= b1). A window may hold two segments — the tail of one sentence and the head of
// the next — with BRK holding the bit of the second segment's first lane (0: one segment);
// units never cross it. tail_known: the byte after lane 63 is past the end of lane 63's sentence.
__device__ WinResult classify_lanes(const Tables& T, const uint32_t* s_ascii,
                                    const uint8_t* __restrict__ text, int64_t i, int64_t b1,
                                    uint32_t byte, uint64_t BRK, bool tail_known) {
  const int lane = lane_id();
  const bool in = i < b1;
  // ASCII bytes for every lane without a branch (beyond the sentence: a separator); the
  // non-ASCII and '[' lanes are revisited only in windows that have them (wave-uniform tests,
  // so a plain window runs no exec-mask branches here)
  const uint32_t ascii_e = s_ascii[byte & 127u];  // (read by every lane: no branch)
  uint32_t cls = in ? ascii_e >> 30 : kSpace;
  int cplen = 1;          // bytes of the code point starting here (0: covered continuation)
  int spk = -1;           // literal special token starting here
  bool slow = in && cls == kDrop;  // non-ASCII or dropped char: not for the register fast path
  bool cont = false;
  if (ballot(in && byte >= 0x80)) {
    if (in && byte >= 0xC0) {
      int64_t j = i;
      const uint32_t cp = utf8_next(text, b1, j);
      cplen = (int)(j - i);
      cls = tab_entry(T, cp) >> 30;
      slow = true;
    } else if (in && byte >= 0x80) {
      cont = true;  // resolved below: covered by a valid lead, or a lone byte (U+FFFD, drop)
      cls = kDrop;
      slow = true;
    }
  }
  if (ballot(in && byte == '[')) {
    if (in && byte == '[') spk = match_special_at(T, text, i, b1);
  }
  const uint64_t V2 = ballot(cplen == 2), V3 = ballot(cplen == 3), V4 = ballot(cplen == 4);
  bool cp_last = cplen <= 1;
  if (V2 | V3 | V4) {  // multi-byte code points in the window (wave-uniform branch)
    const uint64_t C1 = (V2 | V3 | V4) << 1, C2 = (V3 | V4) << 2, C3 = V4 << 3;
    const bool covered = cont && (((C1 | C2 | C3) >> lane) & 1ull);
    const int dist = !covered ? 0 : ((C1 >> lane) & 1ull) ? 1 : ((C2 >> lane) & 1ull) ? 2 : 3;
    // a covered continuation inherits its lead's class; cp_last marks a code point's last byte
    const int lead_len = __shfl((int)(cls | ((uint32_t)cplen << 4)), lane - dist, 64);
    if (covered) {
      cls = (uint32_t)lead_len & 3u;
      cplen = 0;
    }
    cp_last = covered ? (dist == (lead_len >> 4) - 1) : (cplen <= 1);
  }
  const uint64_t S = ballot(spk >= 0), S6 = ballot(spk == kMask);
  const uint64_t inside = (S << 1) | (S << 2) | (S << 3) | (S << 4) | (S6 << 5);
  const bool in_sp = ((S | inside) >> lane) & 1ull;
  const uint32_t cat = in_sp ? kCatSpecial : cls == kSpace ? kCatSep : cls == kIso ? kCatIso : kCatRun;
  const uint64_t RUN = ballot(cat == kCatRun);
  const uint64_t LEAD = ballot(cplen > 0);
  const uint64_t ISO = ballot(cat == kCatIso);
  const uint64_t CPL = ballot(cp_last);
  WinResult R;
  R.slow = ballot(slow);
  R.fallback = false;
  R.ukind = spk >= 0 ? 2 + spk : cat == kCatIso ? 1 : 0;
  R.unit_byte = cat != kCatSep;
  const uint64_t US = S | (ISO & LEAD) | (RUN & ~((RUN << 1) & ~BRK));
  uint64_t RE = RUN & ~((RUN >> 1) & ~(BRK >> 1));
  if (!tail_known) RE &= ~(1ull << 63);
  const uint64_t UE = ((S & ~S6) << 4) | (S6 << 5) | (ISO & CPL & ~inside) | RE;
  R.US = US;
  R.UE = UE;
  R.n_units = __popcll(UE);
  const int n_starts = __popcll(US);
  if (n_starts > R.n_units) {
    const int last = 63 - __clzll(US);
    if (last == 0) {  // a unit of >= 64 bytes
      R.fallback = true;
      R.next_lane = -1;
      return R;
    }
    R.next_lane = last;
  } else if (tail_known) {
    R.next_lane = -1;
  } else {
    // a separator code point straddling the window end restarts the next window at its lead
    const int hl = 63 - __clzll(LEAD);
    const int hc = 63 - __clzll(CPL);
    R.next_lane = hl > hc ? hl : 64;
  }
  return R;
}

// One-sentence window [pos, pos + 64) of a sentence ending at b1; byte = text[pos + lane].
__device__ WinResult classify_window(const Tables& T, const uint32_t* s_ascii,
                                     const uint8_t* __restrict__ text, int64_t pos, int64_t b1,
                                     uint32_t byte) {
  WinResult R = classify_lanes(T, s_ascii, text, pos + lane_id(), b1, byte, 0ull, pos + 64 >= b1);
  R.next = R.next_lane < 0 ? b1 : pos + R.next_lane;
  return R;
}

// The window's units as arrays (W.us / W.ue / W.uk, unit k at index k) for the per-sentence
// kernel, which gives one unit to each lane.
template <typename WL>
__device__ inline void store_units(const WinResult& R, WL& W) {
  const int lane = lane_id();
  if ((R.US >> lane) & 1ull) {
    const int k = (int)popc_below(R.US);
    W.us[k] = (uint8_t)lane;
    W.uk[k] = (uint8_t)R.ukind;
  }
  if ((R.UE >> lane) & 1ull) W.ue[popc_below(R.UE)] = (uint8_t)lane;
  wave_sync();
}

// 32 bytes of text from byte `start` (unaligned); bytes at or past `n_bytes` read as 0 and are
// never loaded.
__device__ inline B32 load32(const uint8_t* __restrict__ text, int64_t n_bytes, int64_t start) {
  const int64_t a = start & ~(int64_t)3;
  const int r = (int)(start & 3);
  uint32_t d[9];
  if (a + 36 <= n_bytes) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(text + a);
#pragma unroll
    for (int k = 0; k < 9; ++k) d[k] = p[k];
  } else {
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      uint32_t v = 0;
      for (int q = 0; q < 4; ++q)
        if (a + 4 * k + q < n_bytes) v |= (uint32_t)text[a + 4 * k + q] << (8 * q);
      d[k] = v;
    }
  }
  uint32_t o[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], r);
  return B32{(uint64_t)o[0] | ((uint64_t)o[1] << 32), (uint64_t)o[2] | ((uint64_t)o[3] << 32),
             (uint64_t)o[4] | ((uint64_t)o[5] << 32), (uint64_t)o[6] | ((uint64_t)o[7] << 32)};
}

__device__ inline uint64_t swar_lower(uint64_t v) {  // A-Z -> a-z on ASCII bytes
  const uint64_t k3f = 0x3f3f3f3f3f3f3f3full, k25 = 0x2525252525252525ull,
                 k80 = 0x8080808080808080ull;
  return v | ((((v + k3f) & ~(v + k25)) & k80) >> 2);
}

// Pieces of one pre-tokenizer unit (text[start, start+len), kind as classify_window): written to
// pc[64 * q]; returns the count, or -1 when the unit needs the lane kernel (> kPcs pieces or a
// normalised word > kNorm bytes). cs_flag: the unit is a literal [CLS] / [SEP].
// ASCII units (words and isolated punctuation, <= 32 bytes) go straight to registers; others are
// normalised code point by code point into the lane's LDS buffer first (ASCII table in LDS).
__device__ int unit_pieces(const Tables& T, const uint32_t* bloom, const uint32_t* s_ascii,
                           const uint8_t* __restrict__ text, int64_t n_bytes, int64_t start,
                           int len, int kind, bool unit_slow, Pcs& pc, uint8_t* w,
                           bool& cs_flag) {
  cs_flag = false;
  if (kind >= 2) {
    pc.put(0, T.special_id[kind - 2]);
    cs_flag = kind - 2 == kCls || kind - 2 == kSep;
    return 1;
  }
  if (!unit_slow && len <= 32 && T.ascii_mode != 0) {
    B32 v = load32(text, n_bytes, start);
    if (T.ascii_mode == 1) v = B32{swar_lower(v.w0), swar_lower(v.w1), swar_lower(v.w2), swar_lower(v.w3)};
    return wordpiece32(T, bloom, v, len, ~0ull, pc);
  }
  // generic (rare): normalise the unit's code points into the lane's LDS buffer
  int nb = 0;
  int64_t j = start;
  const int64_t je = start + len;
  while (j < je) {
    const uint32_t b0 = text[j];
    uint32_t cp, e;
    if (b0 < 0x80) {
      cp = b0;
      e = s_ascii[b0];
      ++j;
    } else {
      cp = utf8_next(text, je, j);
      e = tab_entry(T, cp);
    }
    if ((e >> 30) == kDrop) continue;
    uint8_t ob[12];
    int olen;
    if (e & kIdent) olen = put_utf8(ob, cp);
    else if (e & kMulti) {
      const uint8_t* p = T.pool + (e & 0xFFFFFFu);
      olen = p[0];
      for (int q = 0; q < olen; ++q) ob[q] = p[2 + q];
    } else olen = put_utf8(ob, e & 0x1FFFFFu);
    if (nb + olen > kNorm) return -1;
    for (int q = 0; q < olen; ++q) w[nb + q] = ob[q];
    nb += olen;
  }
  if (nb == 0) return 0;
  // <= 32 normalised bytes (<= 32 chars, so the 100-char rule cannot apply); pieces may end
  // only at character boundaries
  uint64_t ends = 1ull << nb;
  for (int e = 1; e < nb; ++e)
    if ((w[e] & 0xC0) != 0x80) ends |= 1ull << e;
  const uint64_t* w8 = reinterpret_cast<const uint64_t*>(w);
  const B32 v{w8[0], w8[1], w8[2], w8[3]};
  return wordpiece32(T, bloom, v, nb, ends, pc);
}

// The normalised word of a word / isolated-char unit in registers (<= 32 bytes) and the byte
// positions where a piece may end. status: 0 ok, 1 empty (every char dropped: 0 pieces), -1 the
// unit needs the lane kernel (> kNorm normalised bytes). ASCII units are loaded straight from the
// text (SWAR lowercase); others are normalised through the lane's LDS row `w` first.
struct UnitWord {
  B32 v;
  int nb;
  uint64_t ends;
  int status;
};

__device__ UnitWord unit_word(const Tables& T, const uint32_t* s_ascii, const uint8_t* __restrict__ text,
                              int64_t n_bytes, int64_t start, int len, bool unit_slow, uint8_t* w) {
  UnitWord u;
  u.status = 0;
  if (!unit_slow && len <= 32 && T.ascii_mode != 0) {
    B32 v = load32(text, n_bytes, start);
    if (T.ascii_mode == 1) v = B32{swar_lower(v.w0), swar_lower(v.w1), swar_lower(v.w2), swar_lower(v.w3)};
    u.v = v;
    u.nb = len;
    u.ends = ~0ull;
    return u;
  }
  int nb = 0;
  int64_t j = start;
  const int64_t je = start + len;
  while (j < je) {
    const uint32_t b0 = text[j];
    uint32_t cp, e;
    if (b0 < 0x80) {
      cp = b0;
      e = s_ascii[b0];
      ++j;
    } else {
      cp = utf8_next(text, je, j);
      e = tab_entry(T, cp);
    }
    if ((e >> 30) == kDrop) continue;
    uint8_t ob[12];
    int olen;
    if (e & kIdent) olen = put_utf8(ob, cp);
    else if (e & kMulti) {
      const uint8_t* p = T.pool + (e & 0xFFFFFFu);
      olen = p[0];
      for (int q = 0; q < olen; ++q) ob[q] = p[2 + q];
    } else olen = put_utf8(ob, e & 0x1FFFFFu);
    if (nb + olen > kNorm) {
      u.status = -1;
      return u;
    }
    for (int q = 0; q < olen; ++q) w[nb + q] = ob[q];
    nb += olen;
  }
  u.nb = nb;
  if (nb == 0) {
    u.status = 1;
    return u;
  }
  uint64_t ends = 1ull << nb;
  for (int e = 1; e < nb; ++e)
    if ((w[e] & 0xC0) != 0x80) ends |= 1ull << e;
  u.ends = ends;
  const uint64_t* w8 = reinterpret_cast<const uint64_t*>(w);
  u.v = B32{w8[0], w8[1], w8[2], w8[3]};
  return u;
}

__global__ void __launch_bounds__(64 * kTW) tokenize_wave_kernel(
    Tables T, const uint8_t* __restrict__ text, int64_t n_bytes, const int64_t* __restrict__ sent_off,
    int64_t n_sent, int32_t max_pieces, int32_t* __restrict__ ids, int32_t* __restrict__ sent_len,
    int32_t* __restrict__ fb_list, uint32_t* __restrict__ fb_n) {
  __shared__ uint32_t s_ascii[128];
  __shared__ WaveLds s_w[kTW];
  for (int c = threadIdx.x; c < 128; c += blockDim.x) s_ascii[c] = tab_entry(T, (uint32_t)c);
  __syncthreads();
  const int lane = lane_id();
  WaveLds& W = s_w[threadIdx.x >> 6];
  const int64_t stride = (int64_t)gridDim.x * kTW;
  for (int64_t s = (int64_t)blockIdx.x * kTW + wave_id(); s < n_sent; s += stride) {
    const int64_t b0 = sent_off[s], b1 = sent_off[s + 1];
    int64_t pos = b0;
    int32_t emitted = 0, flags = 0;
    bool fallback = false;
    while (pos < b1 && emitted < max_pieces) {
      const uint32_t byte = pos + lane < b1 ? text[pos + lane] : 0x20u;
      const WinResult R = classify_window(T, s_ascii, text, pos, b1, byte);
      if (R.fallback) { fallback = true; break; }
      store_units(R, W);
      int npc = 0;
      bool cs_flag = false;
      Pcs pc{W.pcs + lane};
      if (lane < R.n_units) {
        const int us = W.us[lane], ue = W.ue[lane], kind = W.uk[lane];
        const int ulen = ue - us + 1;
        const bool unit_slow = ((R.slow >> us) & (ulen >= 64 ? ~0ull : ((1ull << ulen) - 1))) != 0;
        npc = unit_pieces(T, T.bloom, s_ascii, text, n_bytes, pos + us, ulen, kind, unit_slow, pc,
                          W.nrm + lane * kNorm, cs_flag);
      }
      if (ballot(npc < 0)) { fallback = true; break; }
      const int incl = wave_incl_scan(npc);
      const int o = emitted + incl - npc;
      for (int q = 0; q < npc; ++q)
        if (o + q < max_pieces) ids[b0 + o + q] = pc.get(q);
      if (ballot(cs_flag && o < max_pieces)) flags = kLenHasClsSep;
      emitted += __shfl(incl, 63, 64);
      pos = R.next;
      wave_sync();
    }
    if (fallback) {
      if (lane == 0) fb_list[atomicAdd(fb_n, 1u)] = (int32_t)s;
    } else if (lane == 0) {
      sent_len[s] = (emitted < max_pieces ? emitted : max_pieces) | flags;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Streaming batched tokenizer (the product path).
//
// A wave claims chunks of kChunk consecutive sentences. Their text is one contiguous byte range
// [A, A + span), which the wave streams in 64-byte banks, one byte per lane, at fixed positions:
// a unit may span banks, so nothing is re-read. Sentence starts inside a bank are break bits
// (BRK); units never cross them. Per bank, ballots give two masks:
//   UNIT  bytes that belong to a pre-tokenizer unit (not a separator, inside the chunk)
//   CONT  bytes that continue the unit of the byte before: the same word run (no break between),
//         a continuation byte of an isolated char, the rest of a literal special token
// Unit starts are UNIT & ~CONT; unit ends are UNIT & ~(CONT >> 1), which needs the next bank's
// first CONT bit, so ends are enqueued one bank late. Starts (chunk-relative byte | kind | slow
// flag) and ends go to two LDS queues in byte order: the k-th start and the k-th end are unit k.
// Banks of plain ASCII (no byte >= 0x80, no control char, no '[', no special token carried in)
// take the short path: one LDS class lookup and three compares per lane. The others take the
// per-code-point classification (UTF-8 leads and continuations, literal specials, the Unicode
// class table) with carries into the next bank.
// Every kSF complete units are resolved in two phases:
//   A (one lane per unit, 64 at a time): literal specials, and one full-length vocab probe of
//     every ASCII word / punctuation unit. ~3/4 of the units are a single piece and are done.
//   B (one lane per unit, 64 at a time): greedy longest-match WordPiece of the remaining "hard"
//     units only (multi-piece words, non-ASCII), deferred across kSF units so that every lane of
//     a phase-B pass has a hard unit.
// Pieces are placed in queue order by a segmented scan over sentences (a unit's sentence by binary
// search of the chunk's sentence starts in LDS). At the end of a chunk the remaining units are
// resolved and every sentence's length (or its fallback) is written.
// Round 2's design re-started a 64-byte window at the last unit start of the window before and
// kept a ring of in-flight sentences; its per-window bookkeeping was ~half of the kernel's
// instructions (profiles/r03l_pmc_tokenizer_variants.txt).
// ---------------------------------------------------------------------------------------------
//
// Word memo (round 6; 19.27 -> 15.25 ms per 2 GB, profiles/r06l_*, r06m_*). Phase B (greedy
// longest match of the multi-piece and non-ASCII words) is
// ~half of the kernel's wave cycles, and its words repeat: in the synthetic corpus 26 % of the
// pre-tokenizer units are multi-piece, and 95 % of those occurrences are words already seen in
// the first 3 % of the text (Zipf). lddl_tokenize therefore runs the kernel twice per call: over
// a leading sample of the sentences (kMemoBuild: every resolved multi-piece word's pieces go to a
// device table, one slot per hash, the first writer claims it by CAS), then over the rest
// (kMemoLookup: a phase-B lane reads its word's slot — one 64-byte entry, normalised bytes as the
// key — and runs the greedy match only on a miss). The table belongs to the call: it is cleared
// before the sample pass, and the two launches order every write before every read, so an entry
// is always one complete (word, pieces) record. The pieces are a function of the normalised word
// alone, so the output is the same with or without the memo (tests run both).
// ---------------------------------------------------------------------------------------------
enum : int { kMemoOff = 0, kMemoBuild = 1, kMemoLookup = 2 };
// 4 M entries x 64 B = 256 MiB (2 M: 15.49 ms per 2 GB, 1 M: 15.83, 4 M: 15.25 — fewer words
// lose their slot to another; profiles/r06m_tok_memo_tuning.txt)
constexpr int kMemoLog2 = 22;
// the sample: 1/32 of the sentences (1/8: 16.06 ms per 2 GB, 1/16: 15.68, 1/64: 15.83)
constexpr int kMemoDiv = 32;
struct WordMemo {
  uint4* tab;  // entry e: tab[4e], tab[4e+1] key bytes 0..31 (zero past nb), tab[4e+2] pieces
               // (8 x uint16), tab[4e+3].x meta: kMemoReady | nb | npc << 8 (0: empty)
  uint32_t mask;
};
constexpr uint32_t kMemoReady = 1u << 31, kMemoClaim = 1u << 30;
__device__ inline B32 memo_key(const B32& v, int nb) {
  return B32{keep_bytes(v.w0, nb), keep_bytes(v.w1, nb - 8), keep_bytes(v.w2, nb - 16),
             keep_bytes(v.w3, nb - 24)};
}
__device__ inline uint32_t memo_slot(const B32& k, int nb) {
  uint64_t h = k.w0 * 0x9E3779B97F4A7C15ull ^ (uint64_t)nb;
  h = (h ^ (h >> 29) ^ k.w1) * 0xBF58476D1CE4E5B9ull;
  h = (h ^ (h >> 32) ^ k.w2) * 0x94D049BB133111EBull;
  h = (h ^ (h >> 29) ^ k.w3) * 0x9E3779B97F4A7C15ull;
  return (uint32_t)(h >> 32);
}

constexpr int kSF = 192;   // units resolved per pass (kSF / 64 phase-A rounds)
// queue capacity: before a bank < kSF complete units; a bank adds <= 64 ends and leaves <= 65
// units open (started, end not yet enqueued)
constexpr int kQ = kSF + 128;
constexpr int kBW = 16;   // waves per workgroup (one workgroup per CU shares the Bloom filter)
constexpr int kChunk = 128;  // consecutive sentences claimed at a time
static_assert((kChunk & (kChunk - 1)) == 0, "binary search over the chunk's sentences");
using HIdx = std::conditional_t<(kSF > 256), uint16_t, uint8_t>;
constexpr int32_t kHardBit = INT32_MIN;  // q_res: pieces are in column (res & 63) of pcs
// q_s entry: chunk-relative start byte (bits 0..27) | kind (28..30: 0 word / isolated char,
// 2 + k literal special k) | kQSlow (the unit holds a byte the register fast path cannot take)
constexpr int32_t kQPos = (1 << 28) - 1;
constexpr int32_t kQSlow = INT32_MIN;
constexpr int64_t kMaxSpan = 1 << 28;  // longer chunks go to the lane kernel
// r_cnt: pieces so far (bits 0..28) | kRFb (the sentence goes to the lane kernel) | kLenHasClsSep
constexpr int32_t kRFb = 1 << 29;
constexpr int32_t kRCnt = kRFb - 1;
static_assert(kLenHasClsSep == (1 << 30), "r_cnt flag layout");
// s_cls: fast-path byte classes
enum : uint32_t { kFRun = 0, kFSep = 1, kFIso = 2, kFSlow = 4 };

struct alignas(16) StreamLds {
  int32_t q_s[kQ];          // unit starts (see kQPos)
  int32_t q_e[kQ];          // unit ends (inclusive, chunk-relative)
  uint8_t q_slot[kQ];       // unit start's sentence slot in the chunk (from the bank loop)
  int32_t q_res[kSF];       // phase A/B result: the single piece id, or kHardBit | column
  uint8_t q_npc[kSF];       // pieces of the unit
  HIdx h_idx[kSF];          // queue positions of the hard units, in order
  int32_t s_off[kChunk + 1];  // chunk-relative sentence starts; s_off[n] = the chunk's length
  int32_t r_cnt[kChunk];    // see kRFb
  // lane l's pieces at pcs[64 q + l]; the same bytes hold lane l's normalised word (32 B at
  // byte 32 l) while phase B loads it into registers, before any piece is written
  alignas(16) int32_t pcs[kPcs * 64];
};
static_assert(kPcs * 64 * 4 >= 64 * kNorm, "normalised-word rows must fit the piece columns");

#ifdef LDDL_STAMPS
__device__ unsigned long long* g_tok_tl;  // diagnostic build: [wave][2] s_memrealtime start / end
// diagnostic build: shader cycles per region, summed over waves (kTokRegions entries)
__device__ unsigned long long* g_tok_reg;
constexpr int kTokRegions = 6;  // 0 banks, 1 phase A, 2 phase B, 3 place, 4 queue shift, 5 chunk
#define TOK_STAMP(r)                                                     \
  do {                                                                   \
    const unsigned long long _now = __builtin_amdgcn_s_memtime();       \
    reg_acc[r] += _now - reg_last;                                       \
    reg_last = _now;                                                     \
  } while (0)
#else
#define TOK_STAMP(r) \
  do {               \
  } while (0)
#endif

template <int kMemo>  // kMemoOff / kMemoBuild / kMemoLookup (word memo above)
__global__ void __launch_bounds__(64 * kBW, 1) tokenize_batch_kernel(
    Tables T_arg, const uint8_t* __restrict__ text, int64_t n_bytes, const int64_t* __restrict__ sent_off,
    int64_t n_sent, int32_t max_pieces, int32_t* __restrict__ ids, int32_t* __restrict__ sent_len_arg,
    int32_t* __restrict__ fb_list_arg, uint32_t* __restrict__ fb_n_arg, int32_t* __restrict__ chunk_ctr_arg,
    WordMemo M) {
  __shared__ uint32_t s_ascii[128];
  __shared__ uint8_t s_cls[256];
  __shared__ uint32_t s_bloom[kBloomWords];
  __shared__ StreamLds s_w[kBW];
  // the tables' pointers and scalars live in LDS, read where used: as kernel arguments they held
  // ~26 SGPRs for the kernel's whole life and pushed the bank loop's own scalars into spills
  __shared__ Tables s_T;
  // (and the per-chunk / rare output pointers, for the same reason)
  __shared__ int32_t* s_cold[4];
  if (threadIdx.x == 0) {
    s_T = T_arg;
    s_cold[0] = sent_len_arg;
    s_cold[1] = fb_list_arg;
    s_cold[2] = reinterpret_cast<int32_t*>(fb_n_arg);
    s_cold[3] = chunk_ctr_arg;
  }
  __syncthreads();
  const Tables& T = s_T;
  int32_t* const volatile* cold = s_cold;  // read where used (not hoisted into registers)
#ifdef LDDL_STAMPS
  const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long reg_acc[kTokRegions] = {0, 0, 0, 0, 0, 0};
  unsigned long long reg_last = __builtin_amdgcn_s_memtime();
  TokStats tstat;
  for (int q = 0; q < 10; ++q) tstat.c[q] = 0;
  TokStats* tsp = &tstat;
#else
  TokStats* tsp = nullptr;
#endif
  for (int c = threadIdx.x; c < 128; c += blockDim.x) s_ascii[c] = tab_entry(T, (uint32_t)c);
  for (int c = threadIdx.x; c < 256; c += blockDim.x) {
    uint32_t v = kFSlow;  // bytes >= 0x80, '[', and the ASCII chars the normaliser drops
    if (c < 128 && c != '[') {
      const uint32_t cl = tab_entry(T, (uint32_t)c) >> 30;
      v = cl == kSpace ? kFSep : cl == kIso ? kFIso : cl == kWord ? kFRun : kFSlow;
    }
    s_cls[c] = (uint8_t)v;
  }
  for (int c = threadIdx.x; c < kBloomWords; c += blockDim.x) s_bloom[c] = T.bloom[c];
  __syncthreads();
  const int lane = lane_id();
  StreamLds& W = s_w[threadIdx.x >> 6];
  // target of the bank loop's lanes that store nothing (no exec-mask branch): the piece columns,
  // unused outside a flush
  int32_t* const trashp = &W.pcs[lane_id()];
  // sentence indices fit int32 (lddl_tokenize: n_sent < INT32_MAX - 2^22)
  const int32_t n_sent32 = (int32_t)n_sent;
  // Chunks: wave w starts with chunk w, then takes the next unclaimed chunk from chunk_ctr
  // (initialised to the number of waves x kChunk). A static share per wave would leave a long
  // tail: waves of one SIMD are issued oldest first, so the first finishes ~25 % before the last.
  int32_t c0;
  {
    const int64_t w = (int64_t)blockIdx.x * kBW + (threadIdx.x >> 6);
    // (readfirstlane: the compiler cannot see that threadIdx.x >> 6 is wave-uniform, and a
    // divergent c0 made the chunk's span, sentence count and every loop over them exec-masked)
    c0 = __builtin_amdgcn_readfirstlane(w * kChunk < n_sent32 ? (int32_t)(w * kChunk) : n_sent32);
  }
  const uint64_t upto = (2ull << lane) - 1;  // lanes <= this one (lane 63: all)

  while (c0 < n_sent32) {
    const int32_t n = n_sent32 - c0 < kChunk ? n_sent32 - c0 : kChunk;
    const int64_t A = sent_off[c0];
    const int64_t span64 = sent_off[c0 + n] - A;
    if (span64 >= kMaxSpan) {  // pathological chunk (>= 256 MiB of text): the lane kernel
      for (int j = lane; j < n; j += 64)
        cold[1][atomicAdd(reinterpret_cast<uint32_t*>(cold[2]), 1u)] = c0 + j;
    } else {
      for (int j = lane; j <= n; j += 64) W.s_off[j] = (int32_t)(sent_off[c0 + j] - A);
      for (int j = lane; j < n; j += 64) W.r_cnt[j] = 0;
      wave_sync();
      const uint32_t span = (uint32_t)span64;
      const uint8_t* __restrict__ ctext = text + A;

      // the sentence holding chunk-relative byte st (the last one starting at or before it: empty
      // sentences at the same offset are skipped)
      auto sent_of = [&](int32_t st) -> int {
        int j = 0;
#pragma unroll
        for (int step = kChunk / 2; step >= 1; step >>= 1) {
          const int k = j + step;
          j = W.s_off[k < n ? k : n] <= st ? k : j;  // s_off[n] = span > st
        }
        return j;
      };

      int ns = 0, ne = 0;  // queued unit starts / ends

      // drop the processed units [0, m) from the queue: < 128 starts and < 128 ends remain
      // (read all, then write)
      auto drop = [&](int m) {
        const int rs = ns - m, re = ne - m;
        int32_t a0 = 0, a1 = 0, e0 = 0, e1 = 0;
        uint8_t l0 = 0, l1 = 0;
        if (lane < rs) a0 = W.q_s[m + lane], l0 = W.q_slot[m + lane];
        if (lane + 64 < rs) a1 = W.q_s[m + 64 + lane], l1 = W.q_slot[m + 64 + lane];
        if (lane < re) e0 = W.q_e[m + lane];
        if (lane + 64 < re) e1 = W.q_e[m + 64 + lane];
        wave_sync();
        if (lane < rs) W.q_s[lane] = a0, W.q_slot[lane] = l0;
        if (lane + 64 < rs) W.q_s[64 + lane] = a1, W.q_slot[64 + lane] = l1;
        if (lane < re) W.q_e[lane] = e0;
        if (lane + 64 < re) W.q_e[64 + lane] = e1;
        wave_sync();
        ns = rs;
        ne = re;
      };

      // place queue units [u0, u1) (all resolved) in order: segmented scan per sentence
      auto place = [&](int u0, int u1) {
        for (int r0 = u0; r0 < u1; r0 += 64) {
          const int u = r0 + lane;
          const bool act = u < u1;
          const int uc = act ? u : u0;
          const int32_t qs = W.q_s[uc];
          const int npc = act ? W.q_npc[uc] : 0;
          const int slot = act ? (int)W.q_slot[uc] : -1;
          const int incl = wave_incl_scan(npc);
          const int excl = incl - npc;
          const int prev_slot = wave_prev(slot);
          const uint64_t F = ballot(act && (lane == 0 || slot != prev_slot));
          const int s0 = 63 - __clzll(F & upto);
          const int seg_excl = excl - __shfl(excl, s0, 64);
          const int next_slot = wave_next(slot);
          const bool seg_last = act && (lane == 63 || u + 1 >= u1 || next_slot != slot);
          if (act) {
            const int o = (W.r_cnt[slot] & kRCnt) + seg_excl;
            const int64_t bb = A + W.s_off[slot];
            const int32_t res = W.q_res[u];
            if (res & kHardBit) {
              const int col = res & 63;
              for (int q = 0; q < npc; ++q)
                if (o + q < max_pieces) ids[bb + o + q] = W.pcs[64 * q + col];
            } else if (npc && o < max_pieces) {
              ids[bb + o] = res;
              const int kind = (qs >> 28) & 7;
              if (kind - 2 == kCls || kind - 2 == kSep) atomicOr(&W.r_cnt[slot], kLenHasClsSep);
            }
          }
          wave_sync();
          if (seg_last) W.r_cnt[slot] += seg_excl + npc;  // (count bits only: < 2^28 pieces)
          wave_sync();
        }
      };

      // resolve and place the complete units [0, m), then drop them from the queue
      auto flush = [&](int m) {
        TOK_STAMP(0);
        // phase A: specials and single-piece words
        int nh = 0;
        {  // all rounds' text loads, then all first table loads, then the checks: one latency each
          constexpr int kR = kSF / 64;
          static_assert(kSF % 64 == 0, "phase A rounds");
          bool elig[kR], hardr[kR];
          int lenr[kR];
          int32_t resr[kR];
          B32 vv[kR];
          Probe pr[kR];
#pragma unroll
          for (int r = 0; r < kR; ++r) {
            const int u = 64 * r + lane;
            elig[r] = hardr[r] = false;
            lenr[r] = 0;
            resr[r] = 0;
            if (u < m) {
              const int32_t qs = W.q_s[u];
              const int st = qs & kQPos, kind = (qs >> 28) & 7;
              const int len = W.q_e[u] - st + 1;
              lenr[r] = len;
              if (kind >= 2) {
                resr[r] = T.special_id[kind - 2];
              } else if (qs >= 0 && T.ascii_mode != 0 && len <= T.max_piece_bytes && len <= 32) {
                elig[r] = true;
                vv[r] = load32(text, n_bytes, A + st);
              } else {
                hardr[r] = true;
              }
            }
          }
#pragma unroll
          for (int r = 0; r < kR; ++r)
            if (elig[r]) {
              if (T.ascii_mode == 1)
                vv[r] = B32{swar_lower(vv[r].w0), swar_lower(vv[r].w1), swar_lower(vv[r].w2), swar_lower(vv[r].w3)};
              pr[r] = probe_first(T, vv[r], lenr[r], 0);
            }
#pragma unroll
          for (int r = 0; r < kR; ++r) {
            if (elig[r]) {
              resr[r] = probe_finish(T, vv[r], lenr[r], pr[r]);
              hardr[r] = resr[r] < 0;
            }
            const int u = 64 * r + lane;
            if (u < m && !hardr[r]) {
              W.q_res[u] = resr[r];
              W.q_npc[u] = 1;
            }
            const uint64_t H = ballot(hardr[r]);
            if (hardr[r]) {
              const int k = nh + (int)popc_below(H);
              W.h_idx[k] = (HIdx)u;
              // a probed word that missed: its (lowercased) bytes go to phase-B row k, so the
              // first phase-B pass reads them from LDS instead of loading the text again
              if (elig[r] && k < 64) {
                uint4* row = reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(W.pcs) + 32 * k);
                row[0] = make_uint4((uint32_t)vv[r].w0, (uint32_t)(vv[r].w0 >> 32), (uint32_t)vv[r].w1,
                                    (uint32_t)(vv[r].w1 >> 32));
                row[1] = make_uint4((uint32_t)vv[r].w2, (uint32_t)(vv[r].w2 >> 32), (uint32_t)vv[r].w3,
                                    (uint32_t)(vv[r].w3 >> 32));
              }
            }
            nh += __popcll(H);
          }
        }
        wave_sync();
        TOK_STAMP(1);
        // phase B in chunks of 64 hard units, each chunk placed with the units before the next one
        int placed = 0;
        if (tsp) {
          tsp->wave(8);
          tsp->add(9, lane == 0 ? m : 0);
        }
        for (int h0 = 0; h0 < nh; h0 += 64) {
          const int hn = nh - h0 < 64 ? nh - h0 : 64;
          if (tsp) {
            tsp->wave(0);
            tsp->add(1, lane < hn);
          }
          int u = -1, st = 0;
          UnitWord uw;
          uw.status = 1;
          bool known_miss = false;
          if (lane < hn) {
            u = W.h_idx[h0 + lane];
            const int32_t qs = W.q_s[u];
            st = qs & kQPos;
            const int len = W.q_e[u] - st + 1;
            const bool slow = qs < 0;
            known_miss = !slow && T.ascii_mode != 0 && len <= T.max_piece_bytes && len <= 32;
            if (h0 == 0 && known_miss) {  // phase A left the word in this lane's row
              const uint4* row = reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(W.pcs) + 32 * lane);
              const uint4 r0 = row[0], r1 = row[1];
              uw.v = B32{r0.x | (uint64_t)r0.y << 32, r0.z | (uint64_t)r0.w << 32,
                         r1.x | (uint64_t)r1.y << 32, r1.z | (uint64_t)r1.w << 32};
              uw.nb = len;
              uw.ends = ~0ull;
              uw.status = 0;
            } else {
              uw = unit_word(T, s_ascii, text, n_bytes, A + st, len, slow,
                             reinterpret_cast<uint8_t*>(W.pcs) + 32 * lane);
            }
          }
          wave_sync();  // every normalised word is in registers: the rows become piece columns
          int npc = 0;
          if (lane < hn) {
            Pcs pc{W.pcs + lane};
            if (uw.status == 0) {
              if constexpr (kMemo == kMemoOff) {
                npc = wordpiece32(T, s_bloom, uw.v, uw.nb, uw.ends, pc, known_miss, tsp);
              } else {
                const B32 key = memo_key(uw.v, uw.nb);
                uint4* e = M.tab + 4 * (size_t)(memo_slot(key, uw.nb) & M.mask);
                bool hit = false;
                if constexpr (kMemo == kMemoLookup) {
                  const uint4 k0 = e[0], k1 = e[1], pz = e[2];
                  const uint32_t meta = e[3].x;
                  hit = (meta & kMemoReady) && (int)(meta & 0xFFu) == uw.nb &&
                        ((k0.x | (uint64_t)k0.y << 32) ^ key.w0 | (k0.z | (uint64_t)k0.w << 32) ^ key.w1 |
                         (k1.x | (uint64_t)k1.y << 32) ^ key.w2 | (k1.z | (uint64_t)k1.w << 32) ^ key.w3) == 0;
                  if (hit) {
                    npc = (int)((meta >> 8) & 0xFu);
                    const uint32_t pw[4] = {pz.x, pz.y, pz.z, pz.w};
#pragma unroll
                    for (int q = 0; q < kPcs; ++q)
                      if (q < npc) pc.put(q, (int32_t)((pw[q >> 1] >> (16 * (q & 1))) & 0xFFFFu));
                  }
                }
                if (!hit) npc = wordpiece32(T, s_bloom, uw.v, uw.nb, uw.ends, pc, known_miss, tsp);
                if constexpr (kMemo == kMemoBuild) {
                  // first writer of the slot in this call claims it; no lane of this launch reads
                  if (npc >= 1 && atomicCAS(&e[3].x, 0u, kMemoClaim) == 0u) {
                    uint32_t pw[4] = {0u, 0u, 0u, 0u};
#pragma unroll
                    for (int q = 0; q < kPcs; ++q)
                      if (q < npc) pw[q >> 1] |= ((uint32_t)pc.get(q) & 0xFFFFu) << (16 * (q & 1));
                    e[0] = make_uint4((uint32_t)key.w0, (uint32_t)(key.w0 >> 32), (uint32_t)key.w1,
                                      (uint32_t)(key.w1 >> 32));
                    e[1] = make_uint4((uint32_t)key.w2, (uint32_t)(key.w2 >> 32), (uint32_t)key.w3,
                                      (uint32_t)(key.w3 >> 32));
                    e[2] = make_uint4(pw[0], pw[1], pw[2], pw[3]);
                    e[3].x = kMemoReady | (uint32_t)uw.nb | (uint32_t)npc << 8;
                  }
                }
              }
            } else if (uw.status < 0) {
              npc = -1;
            }
            if (npc < 0) {  // the sentence goes to the lane kernel
              atomicOr(&W.r_cnt[sent_of(st)], kRFb);
              npc = 0;
            }
            W.q_res[u] = kHardBit | lane;
            W.q_npc[u] = (uint8_t)npc;
          }
          wave_sync();
          const int lim = h0 + 64 < nh ? (int)W.h_idx[h0 + 64] : m;
          TOK_STAMP(2);
          place(placed, lim);
          placed = lim;
          TOK_STAMP(3);
        }
        place(placed, m);
        TOK_STAMP(3);
        drop(m);
        TOK_STAMP(4);
      };

      // ---- the chunk's banks ----
      uint64_t UNITp = 0, CONTp = 0;  // the bank before
      uint64_t cin = 0;               // the byte before the bank is a word-run byte
      // slow-path carries into the next bank: code-point coverage of its first lanes (bit k: lane
      // k continues a lead of the bank before, for leads of 2 / 3 / 4 bytes; <= 3 bits each) and
      // special-token bytes (<= 5 bits), packed k1 | k2 << 8 | k3 << 16 | insc << 24 so that the
      // plain-bank test reads one scalar (as four 64-bit masks they were spilled and reloaded
      // every bank); and the (class | cplen << 4) of the bank's lanes 61..63, one byte each
      uint32_t cpack = 0, plcp = 0;
      int32_t jn = 1;  // the next sentence start to mark
      uint32_t nextS = (uint32_t)__builtin_amdgcn_readfirstlane(W.s_off[1]);
      const uint32_t last = span ? span - 1 : 0;
      // software prefetch three banks ahead (clamped into the chunk; bytes past it are unused)
      uint32_t cur = 0x20u, pf1 = 0x20u, pf2 = 0x20u;
      if (span) {
        cur = ctext[(uint32_t)lane < last ? (uint32_t)lane : last];
        pf1 = ctext[64u + lane < last ? 64u + lane : last];
        pf2 = ctext[128u + lane < last ? 128u + lane : last];
      }
      uint32_t x0 = 0;
      for (; x0 < span; x0 += 64) {
        const uint32_t byte = cur;
        const uint32_t v = s_cls[byte];
        cur = pf1;
        pf1 = pf2;
        {
          const uint32_t xq = x0 + 192u + lane;
          pf2 = ctext[xq < last ? xq : last];
        }
        const uint32_t x = x0 + lane;
        const bool in = x < span;
        uint64_t BRK = 0;
        // this lane's sentence slot (the last sentence starting at or before byte x, as sent_of),
        // stored with its unit start so that placement needs no search
        int32_t lslot = jn - 1;
        while (nextS < x0 + 64) {
          BRK |= 1ull << (nextS - x0);
          lslot += (x0 + lane >= nextS) ? 1 : 0;
          ++jn;
          nextS = jn <= n ? (uint32_t)__builtin_amdgcn_readfirstlane(W.s_off[jn]) : 0xFFFFFFFFu;
        }
        const uint64_t VALID = ballot(in);
        uint64_t RUN, UNIT, CONT, SL = 0;
        // unit start: chunk-relative byte | kind << 28
        int32_t sval = (int32_t)x;
        if (!(ballot(v >= kFSlow) | (uint64_t)cpack)) {  // plain ASCII bank
          RUN = ballot(v == kFRun) & VALID;
          UNIT = VALID & ~ballot(v == kFSep);
          CONT = RUN & ((RUN << 1) | cin) & ~BRK;
        } else {
          const uint64_t k1 = cpack & 0xFFu, k2 = (cpack >> 8) & 0xFFu, k3 = (cpack >> 16) & 0xFFu,
                         insc = cpack >> 24;
          // this lane's sentence end: the next break above the lane, else the first sentence start
          // after the bank
          const uint64_t above = BRK & ~upto;
          const uint32_t se = above ? x0 + (uint32_t)(__ffsll((long long)above) - 1)
                                    : (nextS < span ? nextS : span);
          const int64_t i = A + x, b1 = A + se;
          uint32_t cls = in ? s_ascii[byte & 127u] >> 30 : kSpace;
          int cplen = 1;  // bytes of the code point starting here (0: covered continuation)
          int spk = -1;   // literal special token starting here
          bool slow = in && cls == kDrop;
          bool cont = false;
          if (ballot(in && byte >= 0x80)) {
            if (in && byte >= 0xC0) {
              int64_t j = i;
              const uint32_t cp = utf8_next(text, b1, j);
              cplen = (int)(j - i);
              cls = tab_entry(T, cp) >> 30;
              slow = true;
            } else if (in && byte >= 0x80) {
              cont = true;  // covered by a valid lead, or a lone byte (U+FFFD, dropped)
              cls = kDrop;
              slow = true;
            }
          }
          if (ballot(in && byte == '[')) {
            if (in && byte == '[') spk = match_special_at(T, text, i, b1);
          }
          const int32_t val = (int32_t)(cls | ((uint32_t)cplen << 4));
          const uint64_t V2 = ballot(cplen == 2), V3 = ballot(cplen == 3), V4 = ballot(cplen == 4);
          const uint64_t C1 = ((V2 | V3 | V4) << 1) | k1, C2 = ((V3 | V4) << 2) | k2, C3 = (V4 << 3) | k3;
          if (C1 | C2 | C3) {  // code points of more than one byte (wave-uniform branch)
            const bool covered = cont && (((C1 | C2 | C3) >> lane) & 1ull);
            const int dist = !covered ? 0 : ((C1 >> lane) & 1ull) ? 1 : ((C2 >> lane) & 1ull) ? 2 : 3;
            int lead = __shfl(val, lane - dist, 64);
            if (lane < dist)
              lead = (int)((plcp >> (lane - dist == -1 ? 16 : lane - dist == -2 ? 8 : 0)) & 0xFFu);
            if (covered) {  // a covered continuation takes its lead's class
              cls = (uint32_t)lead & 3u;
              cplen = 0;
            }
          }
          const uint64_t S = ballot(spk >= 0), S6 = ballot(spk == kMask);
          const uint64_t inside = (S << 1) | (S << 2) | (S << 3) | (S << 4) | (S6 << 5) | insc;
          const bool in_sp = ((S | inside) >> lane) & 1ull;
          const uint32_t cat = in_sp ? kCatSpecial : cls == kSpace ? kCatSep : cls == kIso ? kCatIso : kCatRun;
          RUN = ballot(cat == kCatRun);
          const uint64_t ISO = ballot(cat == kCatIso), LEAD = ballot(cplen > 0);
          UNIT = ballot(cat != kCatSep);
          CONT = (RUN & ((RUN << 1) | cin) & ~BRK) | (ISO & ~LEAD) | inside;
          sval = (int32_t)(x | ((uint32_t)(spk >= 0 ? 2 + spk : 0) << 28));
          SL = ballot(slow && cat != kCatSep);
          cpack = (uint32_t)((V2 | V3 | V4) >> 63) | (uint32_t)((V3 | V4) >> 62) << 8 |
                  (uint32_t)(V4 >> 61) << 16 |
                  (uint32_t)((S >> 63) | (S >> 62) | (S >> 61) | (S >> 60) | (S6 >> 59)) << 24;
          plcp = (uint32_t)__builtin_amdgcn_readlane(val, 61) | (uint32_t)__builtin_amdgcn_readlane(val, 62) << 8 |
                 (uint32_t)__builtin_amdgcn_readlane(val, 63) << 16;
        }
        // starts of this bank (lanes without one store to their trash slot)
        const uint64_t US = UNIT & ~CONT;
        {
          const uint32_t r = popc_below(US) + (uint32_t)ns;
          const bool st_here = (US >> lane) & 1ull;
          int32_t* dst = st_here ? &W.q_s[r] : trashp;
          *dst = sval;
          // the unit's sentence slot (placement needs no search)
          uint8_t* sd = st_here ? &W.q_slot[r] : reinterpret_cast<uint8_t*>(trashp);
          *sd = (uint8_t)lslot;
        }
        if (SL) {  // slow bytes flag their unit (started in this bank or before)
          if ((SL >> lane) & 1ull) atomicOr(&W.q_s[ns + (int)__popcll(US & upto) - 1], kQSlow);
        }
        ns += (int)__popcll(US);
        // ends of the bank before
        const uint64_t UEp = UNITp & ~((CONTp >> 1) | (CONT << 63));
        {
          const uint32_t r = popc_below(UEp) + (uint32_t)ne;
          int32_t* dst = ((UEp >> lane) & 1ull) ? &W.q_e[r] : trashp;
          *dst = (int32_t)(x - 64u);
        }
        ne += (int)__popcll(UEp);
        cin = RUN >> 63;
        UNITp = UNIT;
        CONTp = CONT;
        if (ne >= kSF) {
          wave_sync();
          flush(kSF);
        }
      }
      {  // the last bank's ends (nothing continues past the chunk)
        const uint64_t UEp = UNITp & ~(CONTp >> 1);
        const uint32_t r = popc_below(UEp) + (uint32_t)ne;
        int32_t* dst = ((UEp >> lane) & 1ull) ? &W.q_e[r] : trashp;
        *dst = (int32_t)(x0 - 64u + lane);
        ne += (int)__popcll(UEp);
      }
      wave_sync();
      TOK_STAMP(0);
      while (ne > 0) flush(ne < kSF ? ne : kSF);
      // the chunk's sentences
      for (int j = lane; j < n; j += 64) {
        const int32_t rc = W.r_cnt[j];
        if (rc & kRFb) {
          cold[1][atomicAdd(reinterpret_cast<uint32_t*>(cold[2]), 1u)] = c0 + j;
        } else {
          const int32_t cnt = rc & kRCnt;
          cold[0][c0 + j] = (cnt < max_pieces ? cnt : max_pieces) | (rc & kLenHasClsSep);
        }
      }
      wave_sync();  // before the next chunk reuses s_off / r_cnt
    }
    TOK_STAMP(5);
    int32_t nc = 0;
    if (lane == 0) nc = atomicAdd(cold[3], kChunk);
    nc = __builtin_amdgcn_readfirstlane(nc);
    c0 = nc < n_sent32 ? nc : n_sent32;
  }
#ifdef LDDL_STAMPS
  if (lane == 0 && g_tok_tl) {
    const int64_t wv = (int64_t)blockIdx.x * kBW + (threadIdx.x >> 6);
    g_tok_tl[2 * wv] = rt0;
    g_tok_tl[2 * wv + 1] = __builtin_amdgcn_s_memrealtime();
  }
  if (lane == 0 && g_tok_reg)
    for (int r = 0; r < kTokRegions; ++r) atomicAdd(g_tok_reg + r, reg_acc[r]);
  if (g_tok_reg)
    for (int q = 0; q < 10; ++q) {
      const uint64_t v = wave_sum(tstat.c[q]);
      if (lane == 0) atomicAdd(g_tok_reg + kTokRegions + q, (unsigned long long)v);
    }
#endif
}

}  // namespace
}  // namespace lddl

using namespace lddl;

extern "C" int lddl_tokenize(lddl_ctx* c, void* stream, const uint8_t* d_text, int64_t n_bytes,
                             const int64_t* d_sent_off, int64_t n_sent, int32_t max_pieces,
                             int32_t* d_ids, int32_t* d_sent_len) {
  if (!c) LDDL_FAIL(-1, "null ctx");
  if (n_sent < 0 || n_bytes < 0 || max_pieces <= 0 || max_pieces > (1 << 24))
    LDDL_FAIL(-1, "bad sizes (max_pieces must be in 1 .. 2^24)");
  if (n_sent >= (int64_t)INT32_MAX - (1 << 22)) LDDL_FAIL(-1, "too many sentences in one call (%lld)", (long long)n_sent);
  if (n_sent == 0) return 0;
  hipStream_t st = as_stream(stream);
  // diagnostics (each run by tests/test_tokenize_gpu.py against the oracle): "lane" = the
  // fallback kernel for the whole input, "wave" = one sentence per wavefront, "fused" = the
  // default, "plain" = the streaming kernel without the word memo. (Round 6's split form — phase B and placement in launches of their own — measured
  // slower and lives on branch ab/tok-split)
  const char* path = getenv("LDDL_TOKENIZE_PATH");
  if (path && !strcmp(path, "lane")) {
    const int64_t grid = std::min<int64_t>((n_sent + kBlock - 1) / kBlock, 65536);
    hipLaunchKernelGGL(tokenize_lane_kernel, dim3((unsigned)grid), dim3(kBlock), 0, st, c->tab,
                       d_text, d_sent_off, n_sent, max_pieces, d_ids, d_sent_len, nullptr, nullptr);
    LDDL_HIP(hipGetLastError());
    return 0;
  }
  if (path && strcmp(path, "wave") && strcmp(path, "fused") && strcmp(path, "plain"))
    LDDL_FAIL(-1, "LDDL_TOKENIZE_PATH must be lane, wave, fused or plain (got %s)", path);
  // fallback list: [0] = count, then sentence indices
  constexpr int kFbHead = 1;
  DevArena::Block fbb;
  // + the batch kernel's chunk counter after the list
  LDDL_HIP(c->arena.take(sizeof(int32_t) * (size_t)(n_sent + kFbHead + 1), st, fbb));
  int32_t* fb = static_cast<int32_t*>(fbb.p);
  int32_t* chunk_ctr = fb + kFbHead + n_sent;
  LDDL_HIP(hipMemsetAsync(fb, 0, sizeof(int32_t) * kFbHead, st));
  int n_cu = 256;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, c->device);
  // grid-stride over sentences with exactly the resident workgroups (a second wave of
  // workgroups would start only when the first finished: a 2x tail)
  int per_cu = 0;
  if (path && !strcmp(path, "wave")) {  // diagnostics: one sentence per wavefront, no batching
    LDDL_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, tokenize_wave_kernel, 64 * kTW, 0));
    const int64_t want = (n_sent + kTW - 1) / kTW;
    const int64_t grid = std::min<int64_t>(want, (int64_t)n_cu * std::max(per_cu, 1));
    hipLaunchKernelGGL(tokenize_wave_kernel, dim3((unsigned)grid), dim3(64 * kTW), 0, st, c->tab,
                       d_text, n_bytes, d_sent_off, n_sent, max_pieces, d_ids, d_sent_len, fb + kFbHead,
                       reinterpret_cast<uint32_t*>(fb));
  } else {
    const int wpb = kBW;  // waves per workgroup
    LDDL_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, tokenize_batch_kernel<kMemoOff>, 64 * wpb, 0));
#ifdef LDDL_STAMPS
    const int64_t grid_max = (int64_t)n_cu * std::max(per_cu, 1);
    unsigned long long* tl = nullptr;
    unsigned long long* rg = nullptr;
    LDDL_HIP(hipMalloc(&tl, 16 * grid_max * wpb));
    LDDL_HIP(hipMemsetAsync(tl, 0, 16 * grid_max * wpb, st));
    LDDL_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_tok_tl), &tl, sizeof(tl), 0, hipMemcpyHostToDevice, st));
    LDDL_HIP(hipMalloc(&rg, 8 * (kTokRegions + 10)));
    LDDL_HIP(hipMemsetAsync(rg, 0, 8 * (kTokRegions + 10), st));
    LDDL_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_tok_reg), &rg, sizeof(rg), 0, hipMemcpyHostToDevice, st));
#endif
    int64_t grid = 0;
    // one launch of the streaming kernel over sentences [s0, s0 + n) (the sentence offsets are
    // absolute, so a sub-range is a pointer offset), then the lane kernel for its fallback list
    auto pass = [&](int64_t s0, int64_t n, int memo, WordMemo M) -> int {
      const int64_t want = (n + 16 * wpb - 1) / (16 * wpb);
      grid = std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)n_cu * std::max(per_cu, 1)));
      // tests: a smaller grid makes small inputs take the dynamic chunk claims
      if (const char* g = getenv("LDDL_TOKENIZE_GRID")) grid = std::max<int64_t>(1, std::min<int64_t>(grid, atoll(g)));
      // the first grid x wpb chunks are taken statically (chunk w by wave w)
      const int64_t first = std::min<int64_t>(grid * wpb * kChunk, (int64_t)INT32_MAX);
      LDDL_HIP(hipMemsetAsync(fb, 0, sizeof(int32_t) * kFbHead, st));
      LDDL_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(chunk_ctr), (int)first, 1, st));
      const void* kfn = memo == kMemoBuild ? (const void*)tokenize_batch_kernel<kMemoBuild>
                      : memo == kMemoLookup ? (const void*)tokenize_batch_kernel<kMemoLookup>
                                            : (const void*)tokenize_batch_kernel<kMemoOff>;
      const int64_t* so = d_sent_off + s0;
      int32_t* sl = d_sent_len + s0;
      int32_t* fl = fb + kFbHead;
      uint32_t* fn = reinterpret_cast<uint32_t*>(fb);
      void* args[] = {&c->tab, (void*)&d_text, &n_bytes, (void*)&so, &n, &max_pieces, &d_ids, &sl,
                      &fl, &fn, &chunk_ctr, &M};
      LDDL_HIP(hipLaunchKernel(kfn, dim3((unsigned)grid), dim3(64 * kBW), args, 0, st));
      const int64_t fgrid = std::min<int64_t>((n + kBlock - 1) / kBlock, (int64_t)n_cu * 2);
      hipLaunchKernelGGL(tokenize_lane_kernel, dim3((unsigned)fgrid), dim3(kBlock), 0, st, c->tab,
                         d_text, so, n, max_pieces, d_ids, sl, fl, reinterpret_cast<const uint32_t*>(fb));
      LDDL_HIP(hipGetLastError());
      return 0;
    };
    // the word memo (above): a leading sample of 1/32 of the sentences (at least kMemoMinSample)
    // builds it, the rest reads it. Off for vocabs whose ids do not fit 16 bits, for inputs too
    // small to repay the second launch, and with LDDL_TOKENIZE_PATH=plain.
    constexpr int64_t kMemoMinSample = 1 << 14;
    int64_t n_sample = std::max<int64_t>(n_sent / kMemoDiv, kMemoMinSample);
    bool memo = c->vocab_size <= 65536 && n_sent >= 4 * kMemoMinSample;
    if (const char* e = getenv("LDDL_TOKENIZE_MEMO_SAMPLE")) {  // tests: the memo on small inputs
      n_sample = atoll(e);
      memo = c->vocab_size <= 65536 && n_sample > 0 && n_sample < n_sent;
    }
    if (path && !strcmp(path, "plain")) memo = false;
    int rc = 0;
    if (!memo) {
      rc = pass(0, n_sent, kMemoOff, WordMemo{nullptr, 0});
    } else {
      DevArena::Block mb;
      const size_t entries = (size_t)1 << kMemoLog2;
      LDDL_HIP(c->arena.take(64 * entries, st, mb));
      LDDL_HIP(hipMemsetAsync(mb.p, 0, 64 * entries, st));
      const WordMemo M{static_cast<uint4*>(mb.p), (uint32_t)(entries - 1)};
      rc = pass(0, n_sample, kMemoBuild, M);
      if (!rc) rc = pass(n_sample, n_sent - n_sample, kMemoLookup, M);
      c->arena.give(mb, st);
    }
    if (rc) {
      c->arena.give(fbb, st);
      return rc;
    }
#ifdef LDDL_STAMPS
    {  // wave timeline (100 MHz real-time clock)
      const int64_t nw = grid * wpb;
      std::vector<unsigned long long> t(2 * nw);
      LDDL_HIP(hipMemcpyAsync(t.data(), tl, 16 * nw, hipMemcpyDeviceToHost, st));
      LDDL_HIP(hipStreamSynchronize(st));
      unsigned long long t0 = ~0ull, t1 = 0;
      std::vector<double> e(nw);
      for (int64_t q = 0; q < nw; ++q) {
        t0 = std::min(t0, t[2 * q]);
        t1 = std::max(t1, t[2 * q + 1]);
      }
      for (int64_t q = 0; q < nw; ++q) e[q] = (t[2 * q + 1] - t0) / 1e5;
      std::sort(e.begin(), e.end());
      const double span = (t1 - t0) / 1e5;
      fprintf(stderr, "[tok timeline] span %.2f ms, wave end ms: min %.2f p10 %.2f p50 %.2f p90 %.2f max %.2f\n",
              span, e[0], e[nw / 10], e[nw / 2], e[nw * 9 / 10], e[nw - 1]);
      const int nb = 40;
      fprintf(stderr, "[tok timeline] waves alive per %.2f ms bin:", span / nb);
      for (int b = 0; b < nb; ++b) {
        const double te = span * (b + 0.5) / nb;
        int64_t alive = 0;
        for (int64_t q = 0; q < nw; ++q) alive += e[q] > te;
        fprintf(stderr, " %lld", (long long)alive);
      }
      fprintf(stderr, "\n");
      LDDL_HIP(hipFree(tl));
      unsigned long long r[kTokRegions + 10];
      LDDL_HIP(hipMemcpy(r, rg, sizeof r, hipMemcpyDeviceToHost));
      const unsigned long long* k = r + kTokRegions;
      fprintf(stderr,
              "[tok phaseB] flushes %llu units %llu | passes %llu lanes/pass %.1f | piece-steps: wave %llu "
              "lane %llu (lane util %.2f) | bloom iters: wave %llu lane-useful %llu (util %.2f, per wave "
              "step %.1f) | probe trips: wave %llu lane %llu (util %.2f)\n",
              k[8], k[9], k[0], (double)k[1] / (k[0] ? k[0] : 1), k[2], k[3],
              (double)k[3] / (64.0 * (k[2] ? k[2] : 1)), k[4], k[5], (double)k[5] / (64.0 * (k[4] ? k[4] : 1)),
              (double)k[4] / (k[2] ? k[2] : 1), k[6], k[7], (double)k[7] / (64.0 * (k[6] ? k[6] : 1)));
      unsigned long long tot = 0;
      for (int q = 0; q < kTokRegions; ++q) tot += r[q];
      static const char* names[kTokRegions] = {"banks", "phaseA", "phaseB", "place", "qshift", "chunk"};
      fprintf(stderr, "[tok regions] wave-cycle shares:");
      for (int q = 0; q < kTokRegions; ++q) fprintf(stderr, " %s %.1f%%", names[q], 100.0 * r[q] / (tot ? tot : 1));
      fprintf(stderr, "\n");
      LDDL_HIP(hipFree(rg));
    }
#endif
  }
  if (path && !strcmp(path, "wave")) {  // the wave kernel's fallback list
    const int64_t fgrid = std::min<int64_t>((n_sent + kBlock - 1) / kBlock, (int64_t)n_cu * 2);
    hipLaunchKernelGGL(tokenize_lane_kernel, dim3((unsigned)fgrid), dim3(kBlock), 0, st, c->tab,
                       d_text, d_sent_off, n_sent, max_pieces, d_ids, d_sent_len, fb + kFbHead,
                       reinterpret_cast<const uint32_t*>(fb));
    LDDL_HIP(hipGetLastError());
  }
  c->arena.give(fbb, st);
  return 0;
}
