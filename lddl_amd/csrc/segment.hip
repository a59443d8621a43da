// Punkt sentence segmentation on the GPU: the reference's `nltk.tokenize.sent_tokenize(text)`
// (lddl/dask/bert/pretrain.py:86) followed by `strip()` + dropping empty sentences (87-88).
//
// nltk's PunktSentenceTokenizer (nltk/tokenize/punkt.py 3.6.5, a third-party dependency of the
// reference) finds candidate contexts with `period_context_re`
//     \S* [.?!] (?= NonWord | \s+ (\S+) )
// (finditer), decides each with `text_contains_sentbreak(context)` (word tokenisation +
// first/second-pass annotation with the trained parameters), cuts slices at the accepted
// contexts and moves closing brackets/quotes across the cut (`_realign_boundaries`).
//
// Structure used here (derivation in DESIGN.md §4):
//  * finditer yields at most one match per whitespace-free run: the match starts at the run's
//    first byte and ends after the LAST sentence-ending char of the run whose lookahead holds;
//  * a lookahead holds at q iff text[q+1] is a NonWord char, or whitespace with some
//    non-whitespace later in the document (q+1 < rstrip end);
//  * the strip() applied by the reference makes inter-sentence whitespace irrelevant, and the
//    BERT tokenizer ignores whitespace, so each sentence is emitted as [boundary_k,
//    boundary_{k+1}) with the gaps attached to the left sentence: the sentence offsets feed
//    lddl_tokenize directly (documents are contiguous, so the last sentence of a document ends
//    where the next document starts).
//  * the realignment of a cut only depends on the bytes after it: boundary = next sentence start
//    + length of a run of closing chars that is followed by whitespace, "--" or the end.
//
// Kernel: one wavefront per document streams 64-byte windows (one byte per lane). Lanes flag
// whitespace (ASCII by a bit test, other code points through the two-level class table) and
// lookahead-qualified sentence enders; ballots give each selected ender its run start; the
// selected lanes then evaluate their context sequentially (rare: ~1 per sentence) and the
// accepted cuts are appended in order (ballot prefix) to a per-document slot range.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>

#include "common.h"
#include "ctx.h"
#include "device.h"
#include "lddl_amd.h"
#include "scan.h"

namespace lddl {
namespace {

enum : uint32_t { kPSpace = 1, kPUpper = 2, kPLower = 4, kPAlnod = 8, kPDigit = 16 };
enum : uint32_t { kKAbbrev = 1, kKStarter = 2, kKOrtho = 3, kKColloc = 4 };
// nltk _ORTHO_* flags
constexpr uint32_t kOBegUc = 2, kOMidUc = 4, kOUnkUc = 8, kOBegLc = 16, kOMidLc = 32, kOUnkLc = 64;
constexpr uint32_t kOUc = kOBegUc | kOMidUc | kOUnkUc, kOLc = kOBegLc | kOMidLc | kOUnkLc;
constexpr int kMaxKey = 255;  // longest parameter key (bytes)

struct PkEnt {  // open-addressing entry; kind 0 = empty
  uint32_t h;
  uint32_t off;  // key bytes in keys[]
  uint16_t la, lb;
  uint8_t kind, value;
  uint16_t pad;
};

struct PunktTab {
  const uint16_t* l1;
  const uint8_t* pages;
  const int32_t* lower;  // (cp, lower) pairs, sorted
  int32_t n_lower;
  const PkEnt* hash;
  uint32_t hmask;
  int32_t n_rec;
  const uint8_t* keys;
};

__host__ __device__ inline uint32_t fnv_step(uint32_t h, uint32_t b) { return (h ^ b) * 0x01000193u; }
__host__ __device__ inline uint32_t key_hash(uint32_t h, uint32_t kind) {
  h ^= kind * 0x9E3779B9u;
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  return h;
}

// ---- character classes ------------------------------------------------------------------------

// Python `\s` / str.isspace() on ASCII: \t \n \v \f \r, \x1c-\x1f, space
__device__ __forceinline__ bool ascii_space(uint32_t c) {
  return c < 64 && ((0x00000001F0003E00ull >> c) & 1ull);
}
__device__ __forceinline__ bool in_mask(uint32_t c, uint64_t lo, uint64_t hi) {
  return c < 64 ? ((lo >> c) & 1ull) : c < 128 ? ((hi >> (c - 64)) & 1ull) : false;
}
__device__ __forceinline__ bool non_word(uint32_t c) {  // [)";}\]*:@'({[?!]
  return in_mask(c, 0x8c00078600000000ull, 0x2800000028000001ull);
}
__device__ __forceinline__ bool word_start_excl(uint32_t c) {  // not in _re_word_start
  return in_mask(c, 0x0c00374c00000000ull, 0x2800000128000001ull);
}
__device__ __forceinline__ bool ortho_punct(uint32_t c) {  // ";:,.!?"
  return in_mask(c, 0x8c00500200000000ull, 0);
}
__device__ __forceinline__ bool sent_end(uint32_t c) { return c == '.' || c == '?' || c == '!'; }
__device__ __forceinline__ bool closing(uint32_t c) {
  return c == '"' || c == '\'' || c == ')' || c == ']' || c == '}';
}

// Text bytes: the wave's LDS slab when the index falls inside it, else global memory.
struct Src {
  const uint8_t* x;
  const uint8_t* lds;
  int64_t lo, hi;
  __device__ __forceinline__ uint32_t operator[](int64_t i) const {
    return (i >= lo && i < hi) ? (uint32_t)lds[i - lo] : (uint32_t)x[i];
  }
};

__device__ __forceinline__ uint32_t props(const PunktTab& t, uint32_t cp) {
  if (cp >= 0x110000u) return 0;
  return t.pages[(uint32_t)t.l1[cp >> 8] * 256u + (cp & 255u)];
}

__device__ __forceinline__ int utf8_len(uint32_t lead) {
  return lead < 0x80 ? 1 : lead < 0xE0 ? 2 : lead < 0xF0 ? 3 : 4;
}

// code point starting at byte i (a lead byte), bounded by e
__device__ inline uint32_t decode(const Src& s, int64_t i, int64_t e, int* len) {
  const uint32_t c = s[i];
  const int n = utf8_len(c);
  *len = n;
  if (n == 1) return c;
  uint32_t v = n == 2 ? (c & 31u) : n == 3 ? (c & 15u) : (c & 7u);
  for (int k = 1; k < n; ++k) v = (v << 6) | (i + k < e ? (s[i + k] & 63u) : 0u);
  return v;
}

// is the code point containing byte i whitespace (Python `\s`)
__device__ inline bool space_at(const PunktTab& t, const Src& s, int64_t i, int64_t b0, int64_t b1) {
  const uint32_t c = s[i];
  if (c < 0x80) return ascii_space(c);
  int64_t j = i;
  while (j > b0 && j > i - 3 && (s[j] & 0xC0u) == 0x80u) --j;
  int len;
  return (props(t, decode(s, j, b1, &len)) & kPSpace) != 0;
}

__device__ inline uint32_t lower_cp(const PunktTab& t, uint32_t cp, uint32_t* second) {
  *second = 0;
  if (cp < 128) return (cp >= 'A' && cp <= 'Z') ? cp + 32 : cp;
  int lo = 0, hi = t.n_lower - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    const uint32_t k = (uint32_t)t.lower[2 * mid];
    if (k == cp) {
      const int32_t v = t.lower[2 * mid + 1];
      if (v < 0) {  // U+0130 -> U+0069 U+0307
        *second = 0x307;
        return 0x69;
      }
      return (uint32_t)v;
    }
    if (k < cp) lo = mid + 1; else hi = mid - 1;
  }
  return cp;
}

__device__ inline int put_utf8(uint32_t v, uint8_t* o, int k) {
  if (k + 4 > kMaxKey + 1) return kMaxKey + 1;  // too long for any key
  if (v < 0x80) {
    o[k++] = (uint8_t)v;
  } else if (v < 0x800) {
    o[k++] = (uint8_t)(0xC0 | (v >> 6));
    o[k++] = (uint8_t)(0x80 | (v & 63));
  } else if (v < 0x10000) {
    o[k++] = (uint8_t)(0xE0 | (v >> 12));
    o[k++] = (uint8_t)(0x80 | ((v >> 6) & 63));
    o[k++] = (uint8_t)(0x80 | (v & 63));
  } else {
    o[k++] = (uint8_t)(0xF0 | (v >> 18));
    o[k++] = (uint8_t)(0x80 | ((v >> 12) & 63));
    o[k++] = (uint8_t)(0x80 | ((v >> 6) & 63));
    o[k++] = (uint8_t)(0x80 | (v & 63));
  }
  return k;
}

// ---- tokens of a context --------------------------------------------------------------------

struct Tok {
  int64_t s, e;       // bytes
  uint32_t c0;        // first code point
  int c0len;
  bool numeric;       // _RE_NUMERIC on the token -> type "##number##"
  bool period_final, sentbreak, abbr, ellipsis;
};

// type text of [s, e) (lowercased) or "##number##", into o; returns length (> kMaxKey: too long)
__device__ inline int type_text(const PunktTab& t, const Src& x, int64_t s, int64_t e, bool numeric,
                                uint8_t* o) {
  if (numeric) {
    const char* n = "##number##";
    for (int k = 0; k < 10; ++k) o[k] = (uint8_t)n[k];
    return 10;
  }
  int k = 0;
  for (int64_t i = s; i < e && k <= kMaxKey;) {
    int len;
    const uint32_t cp = decode(x, i, e, &len);
    uint32_t sec;
    k = put_utf8(lower_cp(t, cp, &sec), o, k);
    if (sec) k = put_utf8(sec, o, k);
    i += len;
  }
  return k;
}

__device__ inline int lookup(const PunktTab& t, uint32_t kind, const uint8_t* a, int la, const uint8_t* b,
                             int lb) {
  if (t.n_rec == 0 || la > kMaxKey || lb > kMaxKey) return -1;
  uint32_t h = 0x811C9DC5u;
  for (int k = 0; k < la; ++k) h = fnv_step(h, a[k]);
  if (kind == kKColloc) {
    h = fnv_step(h, 0x100u);
    for (int k = 0; k < lb; ++k) h = fnv_step(h, b[k]);
  }
  h = key_hash(h, kind);
  for (uint32_t p = h & t.hmask;; p = (p + 1) & t.hmask) {
    const PkEnt en = t.hash[p];
    if (en.kind == 0) return -1;
    if (en.h != h || en.kind != kind || en.la != la || (kind == kKColloc && en.lb != lb)) continue;
    bool eq = true;
    for (int k = 0; k < la && eq; ++k) eq = t.keys[en.off + k] == a[k];
    for (int k = 0; kind == kKColloc && k < lb && eq; ++k) eq = t.keys[en.off + la + k] == b[k];
    if (eq) return en.value;
  }
}

__device__ inline bool is_numeric(const PunktTab& t, const Src& x, int64_t s, int64_t e) {
  int64_t i = s;
  if (i < e && x[i] == '-') ++i;
  if (i < e && (x[i] == '.' || x[i] == ',')) ++i;
  int len;
  if (i >= e || !(props(t, decode(x, i, e, &len)) & kPDigit)) return false;
  i += len;
  while (i < e) {
    const uint32_t c = x[i];
    if (c == ',' || c == '.' || c == '-') {
      ++i;
      continue;
    }
    if (!(props(t, decode(x, i, e, &len)) & kPDigit)) return false;
    i += len;
  }
  return true;
}

// the token's type without a final period (PunktToken.type_no_period)
__device__ inline int type_no_period(const PunktTab& t, const Src& x, const Tok& k, uint8_t* o) {
  const bool strip = !k.numeric && k.period_final && k.e - k.s > 1;
  return type_text(t, x, k.s, k.e - (strip ? 1 : 0), k.numeric, o);
}
__device__ inline int type_no_sentperiod(const PunktTab& t, const Src& x, const Tok& k, uint8_t* o) {
  return k.sentbreak ? type_no_period(t, x, k, o) : type_text(t, x, k.s, k.e, k.numeric, o);
}

__device__ inline void make_tok(const PunktTab& t, const Src& x, int64_t s, int64_t e, Tok& k) {
  k.s = s;
  k.e = e;
  k.c0 = decode(x, s, e, &k.c0len);
  k.numeric = is_numeric(t, x, s, e);
  k.period_final = x[e - 1] == '.';
  k.sentbreak = k.abbr = k.ellipsis = false;
  // _first_pass_annotation
  const int64_t n = e - s;
  if (n == 1 && sent_end(x[s])) {
    k.sentbreak = true;
    return;
  }
  bool dots = n >= 2;
  for (int64_t i = s; i < e && dots; ++i) dots = x[i] == '.';
  if (dots) {
    k.ellipsis = true;
    return;
  }
  if (k.period_final && !(n >= 2 && x[e - 2] == '.')) {
    bool hit = false;
    if (t.n_rec) {  // tok[:-1].lower() or its last '-' component in abbrev_types
      uint8_t buf[kMaxKey + 8];
      const int l = type_text(t, x, s, e - 1, false, buf);
      hit = lookup(t, kKAbbrev, buf, l, nullptr, 0) >= 0;
      if (!hit && l <= kMaxKey) {
        int d = l;
        while (d > 0 && buf[d - 1] != '-') --d;
        if (d > 0) hit = lookup(t, kKAbbrev, buf + d, l - d, nullptr, 0) >= 0;
      }
    }
    if (hit) k.abbr = true; else k.sentbreak = true;
  }
}

// _ortho_heuristic: 1 True, 0 False, 2 unknown
__device__ inline int ortho_heuristic(const PunktTab& t, const Src& x, const Tok& k) {
  if (k.e - k.s == 1 && ortho_punct(x[k.s])) return 0;
  uint32_t oc = 0;
  if (t.n_rec) {
    uint8_t buf[kMaxKey + 8];
    const int l = type_no_sentperiod(t, x, k, buf);
    const int v = lookup(t, kKOrtho, buf, l, nullptr, 0);
    oc = v < 0 ? 0u : (uint32_t)v;
  }
  const uint32_t p = props(t, k.c0);
  if ((p & kPUpper) && (oc & kOLc) && !(oc & kOMidUc)) return 1;
  if ((p & kPLower) && ((oc & kOUc) || !(oc & kOBegLc))) return 0;
  return 2;
}

// _second_pass_annotation of a given its successor b
__device__ inline void second_pass(const PunktTab& t, const Src& x, Tok& a, const Tok& b) {
  if (!a.period_final) return;
  const bool initial = a.e - a.s == a.c0len + 1 && (props(t, a.c0) & kPAlnod);
  uint8_t typ[kMaxKey + 8], nxt[kMaxKey + 8];
  int lt = 0, ln = 0;
  if (t.n_rec) {
    lt = type_no_period(t, x, a, typ);
    ln = type_no_sentperiod(t, x, b, nxt);
    if (lookup(t, kKColloc, typ, lt, nxt, ln) >= 0) {
      a.sentbreak = false;
      a.abbr = true;
      return;
    }
  }
  if ((a.abbr || a.ellipsis) && !initial) {
    if (ortho_heuristic(t, x, b) == 1) {
      a.sentbreak = true;
      return;
    }
    if ((props(t, b.c0) & kPUpper) && t.n_rec && lookup(t, kKStarter, nxt, ln, nullptr, 0) >= 0) {
      a.sentbreak = true;
      return;
    }
  }
  if (initial || a.numeric) {  // typ == "##number##" iff the token is numeric
    const int h = ortho_heuristic(t, x, b);
    if (h == 0) {
      a.sentbreak = false;
      a.abbr = true;
      return;
    }
    if (h == 2 && initial && (props(t, b.c0) & kPUpper)) {
      int v = t.n_rec ? lookup(t, kKOrtho, nxt, ln, nullptr, 0) : -1;
      if (!(v >= 0 && ((uint32_t)v & kOLc))) {
        a.sentbreak = false;
        a.abbr = true;
      }
    }
  }
}

// end-of-word lookahead of _word_tokenize_fmt at e inside a whitespace-free segment ending at se
__device__ inline bool word_end(const Src& x, int64_t e, int64_t se) {
  if (e >= se) return true;
  const uint32_t c = x[e];
  const uint32_t d = e + 1 < se ? x[e + 1] : 0u;
  if (non_word(c) || (c == '-' && d == '-') || (c == '.' && d == '.')) return true;
  if (c == ',') {
    if (e + 1 >= se || non_word(d)) return true;
    const uint32_t f = e + 2 < se ? x[e + 2] : 0u;
    return (d == '-' && f == '-') || (d == '.' && f == '.');
  }
  return false;
}

// next token of the whitespace-free segment [p, se); returns its end
__device__ inline int64_t next_word(const Src& x, int64_t p, int64_t se) {
  const uint32_t c = x[p];
  const uint32_t d = p + 1 < se ? x[p + 1] : 0u;
  if ((c == '-' || c == '.') && d == c) {  // MultiChar \-{2,} | \.{2,}
    int64_t e = p;
    while (e < se && x[e] == c) ++e;
    return e;
  }
  if (word_start_excl(c)) return p + 1;  // \S (ASCII)
  int64_t e = p + 1;  // (?=WordStart)\S+? up to the end lookahead
  while (!word_end(x, e, se)) ++e;
  return e;
}

// text_contains_sentbreak over the context: segment [s1, e1) then (if s2 < e2) [s2, e2)
__device__ inline bool contains_sentbreak(const PunktTab& t, const Src& x, int64_t s1, int64_t e1,
                                          int64_t s2, int64_t e2) {
  Tok cur, nxt;
  int64_t p = s1, se = e1;
  bool have = false;
  while (true) {
    if (p >= se) {
      if (se == e1 && s2 < e2) {
        p = s2;
        se = e2;
      } else {
        break;
      }
    }
    const int64_t e = next_word(x, p, se);
    if (!have) {
      make_tok(t, x, p, e, cur);
      have = true;
    } else {
      make_tok(t, x, p, e, nxt);
      second_pass(t, x, cur, nxt);
      if (cur.sentbreak) return true;
      cur = nxt;
    }
    p = e;
  }
  return false;
}

constexpr int kSegWaves = 4;
constexpr int kSlab = 6144;     // LDS bytes per wave: [blk - kSlabBack, blk + kSlab - kSlabBack)
constexpr int kSlabBack = 256;  // look-behind kept for run starts / contexts
constexpr int kBlk = kSlab - 2 * kSlabBack;  // bytes classified per slab (look-ahead = kSlabBack)
constexpr int kQ = 128;         // queued candidate contexts per wave

// One selected sentence ender q (with the start of its whitespace-free run): evaluate its
// period context, and if it is a cut, its realigned boundary.
template <bool kParams>
__device__ inline bool eval_candidate(const PunktTab& t, const Src& src, int64_t i, int64_t run_start,
                                      int64_t b0, int64_t b1, int64_t rs, int64_t* bound) {
  int64_t s2 = 0, e2 = 0, e1 = i + 1, next_start;
  if (non_word(src[i + 1])) {
    e1 = i + 2;  // context = match + the NonWord char
    next_start = i + 1;
  } else {
    s2 = i + 1;
    while (space_at(t, src, s2, b0, b1)) ++s2;  // non-whitespace exists before rs
    e2 = s2;
    while (e2 < b1 && !space_at(t, src, e2, b0, b1)) ++e2;
    next_start = s2;
  }
  if (!contains_sentbreak(t, src, run_start, e1, s2, e2)) return false;
  // _realign_boundaries: a closing run followed by whitespace, "--" or the end moves left
  int64_t k = next_start;
  while (k < rs && closing(src[k])) ++k;
  const bool ok = k > next_start &&
                  (k >= rs || space_at(t, src, k, b0, b1) || (src[k] == '-' && k + 1 < b1 && src[k + 1] == '-'));
  *bound = ok ? k : next_start;
  return true;
}

// one wavefront per document; rel[] receives the cut positions (relative to the document start)
// at slot base (doc_off[d] - doc_off[0]) / 2 + d, cnt[d] = 1 + number of cuts.
// The document streams through a per-wave LDS slab (16 B per lane per load). Lanes classify one
// byte each per 64-byte window and queue the selected enders (position + run start) in LDS; the
// queue is evaluated one candidate per lane (the sequential context walk reads the slab; bytes
// outside it come from global memory through Src) and the cuts are appended in order.
// kParams = false: the untrained tokenizer (no parameter lookups, no private key buffers)
template <bool kParams>
__global__ void __launch_bounds__(64 * kSegWaves) segment_kernel(PunktTab t, const uint8_t* __restrict__ x,
                                                                  int64_t n_bytes,
                                                                  const int64_t* __restrict__ doc_off,
                                                                  int64_t n_doc, int32_t* __restrict__ rel,
                                                                  int32_t* __restrict__ cnt) {
  __shared__ uint4 slab_all[kSegWaves][kSlab / 16];
  __shared__ int32_t queue_all[kSegWaves][2][kQ];
  const int64_t d = (int64_t)blockIdx.x * kSegWaves + (threadIdx.x >> 6);
  if (d >= n_doc) return;  // wave-uniform
  if (!kParams) t.n_rec = 0;
  const int lane = lane_id();
  uint4* slab = slab_all[threadIdx.x >> 6];
  int32_t* qpos = queue_all[threadIdx.x >> 6][0];
  int32_t* qrun = queue_all[threadIdx.x >> 6][1];
  const int64_t b0 = doc_off[d], b1 = doc_off[d + 1];
  int32_t* out = rel + ((b0 - doc_off[0]) >> 1) + d;
  const Src g{x, reinterpret_cast<const uint8_t*>(slab), 0, 0};  // global only
  // rstrip end: one past the last non-whitespace byte
  int64_t rs = b0;
  for (int64_t we = b1; we > b0; we -= 64) {
    const int64_t i = we - 64 + lane;
    const bool nonsp = i >= b0 && !space_at(t, g, i, b0, b1);
    const uint64_t m = ballot(nonsp);
    if (m) {
      rs = we - 64 + (63 - __builtin_clzll(m)) + 1;
      break;
    }
  }
  const bool aligned = ((uintptr_t)x & 15u) == 0;
  int32_t nb = 0;
  int64_t last_sp = b0 - 1;  // last whitespace byte before the window
  for (int64_t blk = b0; blk < rs; blk += kBlk) {
    // slab [lo, hi): 16-byte aligned, inside the text buffer
    const int64_t lo = std::max<int64_t>(0, (blk - kSlabBack) & ~(int64_t)15);
    const int64_t hi = std::min<int64_t>(n_bytes, lo + kSlab);
    wave_sync();  // previous slab and queue fully consumed
    for (int r = lane; r < kSlab / 16; r += 64) {
      const int64_t a = lo + 16 * (int64_t)r;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (a + 16 <= hi && aligned) {
        v = *reinterpret_cast<const uint4*>(x + a);
      } else if (a < hi) {
        uint8_t tmp[16] = {};
        for (int k = 0; k < 16 && a + k < hi; ++k) tmp[k] = x[a + k];
        memcpy(&v, tmp, 16);
      }
      slab[r] = v;
    }
    wave_sync();
    const Src src{x, reinterpret_cast<const uint8_t*>(slab), lo, hi};
    const int64_t bend = std::min<int64_t>(rs, blk + kBlk);
    int qn = 0;
    for (int64_t base = blk;; base += 64) {
      const bool more = base < bend;
      if (more) {
        const int64_t i = base + lane;
        const bool valid = i < rs;
        const uint32_t c = valid ? src[i] : 0u;
        const bool sp = valid && space_at(t, src, i, b0, b1);
        // lookahead-qualified sentence ender that is the last one of its run
        bool sel = false;
        if (valid && sent_end(c) && i + 1 < rs) {
          const uint32_t cj = src[i + 1];
          if (non_word(cj)) {
            sel = true;  // scan the rest of the run for a later qualified ender
            for (int64_t k = i + 1; k < rs && sel; ++k) {
              if (space_at(t, src, k, b0, b1)) break;
              if (sent_end(src[k]) && k + 1 < rs && (non_word(src[k + 1]) || space_at(t, src, k + 1, b0, b1)))
                sel = false;
            }
          } else {
            sel = space_at(t, src, i + 1, b0, b1);
          }
        }
        const uint64_t spm = ballot(sp);
        const uint64_t below = spm & ((1ull << lane) - 1ull);
        const int64_t run_start = below ? base + (63 - __builtin_clzll(below)) + 1 : last_sp + 1;
        if (spm) last_sp = base + (63 - __builtin_clzll(spm));
        const uint64_t sm = ballot(sel);
        if (sel) {
          const int slot = qn + (int)popc_below(sm);
          qpos[slot] = (int32_t)(i - b0);
          qrun[slot] = (int32_t)(run_start - b0);
        }
        qn += __builtin_popcountll(sm);
      }
      if (qn > kQ - 64 || (!more && qn > 0)) {  // evaluate the queue, one candidate per lane
        wave_sync();
        for (int c0 = 0; c0 < qn; c0 += 64) {
          bool cut = false;
          int64_t bound = 0;
          if (c0 + lane < qn)
            cut = eval_candidate<kParams>(t, src, b0 + qpos[c0 + lane], b0 + qrun[c0 + lane], b0, b1, rs,
                                          &bound);
          const uint64_t cm = ballot(cut);
          if (cut) out[nb + (int32_t)popc_below(cm)] = (int32_t)(bound - b0);
          nb += __builtin_popcountll(cm);
        }
        wave_sync();
        qn = 0;
      }
      if (!more) break;
    }
  }
  if (lane == 0) cnt[d] = nb + 1;
}

struct CntAt {
  const int32_t* cnt;
  __device__ int64_t operator()(int64_t i) const { return cnt[i]; }
};

// sent_off[doc_sent_off[d] + k]: document start, then its cuts; sent_off[n_sent] = text end
__global__ void segment_fill_kernel(const int64_t* __restrict__ doc_off, int64_t n_doc,
                                    const int32_t* __restrict__ rel, const int64_t* __restrict__ dso,
                                    int64_t* __restrict__ sent_off) {
  const int64_t d = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (d >= n_doc) return;
  const int64_t b0 = doc_off[d];
  const int32_t* in = rel + ((b0 - doc_off[0]) >> 1) + d;
  const int64_t o = dso[d], n = dso[d + 1] - o;
  for (int64_t k = lane_id(); k < n; k += 64) sent_off[o + k] = k == 0 ? b0 : b0 + in[k - 1];
  if (d == n_doc - 1 && lane_id() == 0) sent_off[dso[n_doc]] = doc_off[n_doc];
}

}  // namespace
}  // namespace lddl

using namespace lddl;

struct lddl_punkt_state {
  uint16_t* l1 = nullptr;
  uint8_t* pages = nullptr;
  int32_t* lower = nullptr;
  int32_t n_lower = 0;
  PkEnt* hash = nullptr;
  uint32_t hmask = 0;
  int32_t n_rec = 0;
  uint8_t* keys = nullptr;
  // pending segmentation (between lddl_segment_count and lddl_segment_fill)
  DevArena::Block rel, cnt, dso, scratch;
  const int64_t* doc_off = nullptr;
  int64_t n_doc = -1;
  int64_t n_sent = 0;
  void free_tables() {
    (void)hipFree(l1);
    (void)hipFree(pages);
    (void)hipFree(lower);
    (void)hipFree(hash);
    (void)hipFree(keys);
    l1 = nullptr;
    pages = nullptr;
    lower = nullptr;
    hash = nullptr;
    keys = nullptr;
  }
};

static lddl_punkt_state* punkt_of(lddl_ctx* c) {
  return reinterpret_cast<lddl_punkt_state*>(c->punkt);
}

extern "C" void lddl_punkt_release(lddl_ctx* c) {
  lddl_punkt_state* p = punkt_of(c);
  if (!p) return;
  (void)hipDeviceSynchronize();
  p->free_tables();
  for (DevArena::Block* b : {&p->rel, &p->cnt, &p->dso, &p->scratch})
    if (b->p) (void)hipFree(b->p);
  delete p;
  c->punkt = nullptr;
}

extern "C" int lddl_punkt_set_params(lddl_ctx* c, const uint8_t* table, int64_t table_bytes,
                                     const uint8_t* records, int64_t records_bytes) {
  if (!c) LDDL_FAIL(-1, "null ctx");
  if (!table || table_bytes < 16 + 0x1100 * 2 || memcmp(table, "LDPK", 4) != 0)
    LDDL_FAIL(-1, "bad Punkt character table");
  uint32_t hdr[3];
  memcpy(hdr, table + 4, 12);
  const int64_t need = 16 + 0x1100 * 2 + (int64_t)hdr[1] * 256 + (int64_t)hdr[2] * 8;
  if (hdr[0] != 1 || table_bytes < need) LDDL_FAIL(-1, "truncated Punkt character table");
  // parameter records: u8 kind, u8 value, u16 la, u16 lb, a bytes, b bytes
  std::vector<PkEnt> ents;
  std::vector<uint8_t> keys;
  for (int64_t r = 0; r < records_bytes;) {
    if (r + 6 > records_bytes) LDDL_FAIL(-1, "truncated Punkt parameter record");
    const uint8_t* q = records + r;
    PkEnt e{};
    e.kind = q[0];
    e.value = q[1];
    e.la = (uint16_t)(q[2] | (q[3] << 8));
    e.lb = (uint16_t)(q[4] | (q[5] << 8));
    if (e.kind < kKAbbrev || e.kind > kKColloc) LDDL_FAIL(-1, "bad Punkt parameter kind %d", e.kind);
    if (e.la > kMaxKey || e.lb > kMaxKey)
      LDDL_FAIL(-1, "Punkt parameter key longer than %d bytes", kMaxKey);
    if (r + 6 + e.la + e.lb > records_bytes) LDDL_FAIL(-1, "truncated Punkt parameter record");
    uint32_t h = 0x811C9DC5u;
    for (int k = 0; k < e.la; ++k) h = fnv_step(h, q[6 + k]);
    if (e.kind == kKColloc) {
      h = fnv_step(h, 0x100u);
      for (int k = 0; k < e.lb; ++k) h = fnv_step(h, q[6 + e.la + k]);
    }
    e.h = key_hash(h, e.kind);
    e.off = (uint32_t)keys.size();
    keys.insert(keys.end(), q + 6, q + 6 + e.la + e.lb);
    ents.push_back(e);
    r += 6 + e.la + e.lb;
  }
  uint32_t cap = 16;
  while (cap < 2 * ents.size() + 16) cap <<= 1;
  std::vector<PkEnt> tab(cap);
  for (const PkEnt& e : ents) {
    uint32_t p = e.h & (cap - 1);
    bool dup = false;
    while (tab[p].kind) {
      const PkEnt& o = tab[p];
      if (o.h == e.h && o.kind == e.kind && o.la == e.la && o.lb == e.lb &&
          !memcmp(&keys[o.off], &keys[e.off], e.la + e.lb)) {
        dup = true;  // a set: first record wins (ortho_context keys are unique in nltk)
        break;
      }
      p = (p + 1) & (cap - 1);
    }
    if (!dup) tab[p] = e;
  }
  lddl_punkt_state* ps = punkt_of(c);
  if (!ps) {
    ps = new lddl_punkt_state();
    c->punkt = ps;
  }
  LDDL_HIP(hipSetDevice(c->device));
  LDDL_HIP(hipDeviceSynchronize());
  ps->free_tables();
  const size_t l1b = 0x1100 * 2, pgb = (size_t)hdr[1] * 256, lwb = (size_t)hdr[2] * 8;
  LDDL_HIP(hipMalloc(&ps->l1, l1b));
  LDDL_HIP(hipMalloc(&ps->pages, pgb));
  LDDL_HIP(hipMalloc(&ps->lower, std::max<size_t>(lwb, 8)));
  LDDL_HIP(hipMalloc(&ps->hash, sizeof(PkEnt) * cap));
  LDDL_HIP(hipMalloc(&ps->keys, std::max<size_t>(keys.size(), 8)));
  LDDL_HIP(hipMemcpy(ps->l1, table + 16, l1b, hipMemcpyHostToDevice));
  LDDL_HIP(hipMemcpy(ps->pages, table + 16 + l1b, pgb, hipMemcpyHostToDevice));
  if (lwb) LDDL_HIP(hipMemcpy(ps->lower, table + 16 + l1b + pgb, lwb, hipMemcpyHostToDevice));
  LDDL_HIP(hipMemcpy(ps->hash, tab.data(), sizeof(PkEnt) * cap, hipMemcpyHostToDevice));
  if (!keys.empty()) LDDL_HIP(hipMemcpy(ps->keys, keys.data(), keys.size(), hipMemcpyHostToDevice));
  ps->n_lower = (int32_t)hdr[2];
  ps->hmask = cap - 1;
  ps->n_rec = (int32_t)ents.size();
  return 0;
}

extern "C" int lddl_segment_count(lddl_ctx* c, void* stream, const uint8_t* d_text, int64_t n_bytes,
                                  const int64_t* d_doc_off, int64_t n_doc, int64_t* n_sent) {
  if (!c) LDDL_FAIL(-1, "null ctx");
  lddl_punkt_state* ps = punkt_of(c);
  if (!ps || !ps->l1) LDDL_FAIL(-1, "Punkt parameters not set (lddl_punkt_set_params)");
  if (n_doc < 0 || n_bytes < 0 || !n_sent) LDDL_FAIL(-1, "bad sizes");
  if (ps->n_doc >= 0) LDDL_FAIL(-1, "a segmentation is pending: call lddl_segment_fill first");
  hipStream_t st = as_stream(stream);
  const int64_t slots = n_bytes / 2 + n_doc + 2;
  LDDL_HIP(c->arena.take(sizeof(int32_t) * (size_t)slots, st, ps->rel));
  LDDL_HIP(c->arena.take(sizeof(int32_t) * (size_t)(n_doc + 1), st, ps->cnt));
  LDDL_HIP(c->arena.take(sizeof(int64_t) * (size_t)(n_doc + 1), st, ps->dso));
  LDDL_HIP(c->arena.take(sizeof(int64_t) * (size_t)scan_scratch_elems(n_doc), st, ps->scratch));
  int32_t* cnt = static_cast<int32_t*>(ps->cnt.p);
  int64_t* dso = static_cast<int64_t*>(ps->dso.p);
  if (n_doc > 0) {
    PunktTab t{ps->l1, ps->pages, ps->lower, ps->n_lower, ps->hash, ps->hmask, ps->n_rec, ps->keys};
    const int64_t grid = (n_doc + kSegWaves - 1) / kSegWaves;
    if (ps->n_rec)
      hipLaunchKernelGGL(segment_kernel<true>, dim3((unsigned)grid), dim3(64 * kSegWaves), 0, st, t, d_text,
                         n_bytes, d_doc_off, n_doc, static_cast<int32_t*>(ps->rel.p), cnt);
    else
      hipLaunchKernelGGL(segment_kernel<false>, dim3((unsigned)grid), dim3(64 * kSegWaves), 0, st, t, d_text,
                         n_bytes, d_doc_off, n_doc, static_cast<int32_t*>(ps->rel.p), cnt);
    LDDL_HIP(hipGetLastError());
  }
  LDDL_HIP(scan_exclusive(CntAt{cnt}, n_doc, dso, static_cast<int64_t*>(ps->scratch.p), st));
  LDDL_HIP(hipMemcpyAsync(&ps->n_sent, dso + n_doc, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  LDDL_HIP(hipStreamSynchronize(st));
  ps->doc_off = d_doc_off;
  ps->n_doc = n_doc;
  *n_sent = ps->n_sent;
  return 0;
}

extern "C" int lddl_segment_fill(lddl_ctx* c, void* stream, int64_t* d_sent_off, int64_t* d_doc_sent_off) {
  if (!c) LDDL_FAIL(-1, "null ctx");
  lddl_punkt_state* ps = punkt_of(c);
  if (!ps || ps->n_doc < 0) LDDL_FAIL(-1, "no pending segmentation (lddl_segment_count)");
  hipStream_t st = as_stream(stream);
  const int64_t n_doc = ps->n_doc;
  int rc = 0;
  if (n_doc > 0) {
    const int64_t grid = (n_doc + 3) / 4;
    hipLaunchKernelGGL(segment_fill_kernel, dim3((unsigned)grid), dim3(256), 0, st, ps->doc_off, n_doc,
                       static_cast<const int32_t*>(ps->rel.p), static_cast<const int64_t*>(ps->dso.p),
                       d_sent_off);
  } else {
    if (hipMemsetAsync(d_sent_off, 0, sizeof(int64_t), st) != hipSuccess) rc = -100;
  }
  if (hipMemcpyAsync(d_doc_sent_off, ps->dso.p, sizeof(int64_t) * (size_t)(n_doc + 1), hipMemcpyDeviceToDevice,
                     st) != hipSuccess)
    rc = -100;
  if (hipGetLastError() != hipSuccess) rc = -100;
  for (DevArena::Block* b : {&ps->rel, &ps->cnt, &ps->dso, &ps->scratch}) {
    c->arena.give(*b, st);
    *b = DevArena::Block{};
  }
  ps->n_doc = -1;
  if (rc) LDDL_FAIL(rc, "lddl_segment_fill: HIP launch/copy failed");
  return 0;
}
