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
// (Explicit address spaces: a select between the two pointers would become flat loads, which
// wait on both the vector-memory and the LDS counters.)
typedef const __attribute__((address_space(3))) uint8_t* lds_u8_ptr;
typedef const __attribute__((address_space(1))) uint8_t* glb_u8_ptr;
struct Src {
  glb_u8_ptr x;
  lds_u8_ptr lds;
  int64_t lo, hi;
  __device__ Src(const uint8_t* gx, const void* l, int64_t lo_, int64_t hi_)
      : x((glb_u8_ptr)gx), lds((lds_u8_ptr)l), lo(lo_), hi(hi_) {}
  __device__ __forceinline__ uint32_t operator[](int64_t i) const {
    if (i >= lo && i < hi) return lds[i - lo];
    return x[i];
  }
};

// class bits of an ASCII code point, computed (the table agrees: tests/test_punkt.py)
__device__ __forceinline__ uint32_t ascii_props(uint32_t c) {
  const bool up = c - 'A' < 26u, lo = c - 'a' < 26u;
  return (ascii_space(c) ? kPSpace : 0u) | (up ? kPUpper : 0u) | (lo ? kPLower : 0u) |
         ((up || lo || c == '_') ? kPAlnod : 0u) | (c - '0' < 10u ? kPDigit : 0u);
}

__device__ __forceinline__ uint32_t props(const PunktTab& t, uint32_t cp) {
  if (cp < 128u) return ascii_props(cp);
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
  k.period_final = x[e - 1] == '.';
  // the type ("##number##" or not) is only consulted for period-final tokens and parameter keys
  k.numeric = (k.period_final || t.n_rec) ? is_numeric(t, x, s, e) : false;
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
constexpr int kSlab = 4096;     // LDS bytes per classifying wave
constexpr int kCtx = 64;        // context bytes staged per candidate lane
constexpr int kRowW = 17;       // LDS row stride in dwords (68 B: conflict-free byte walks)
constexpr int kEvalBlock = 256;

// One qualified sentence ender q: if it is the match of its run (the last qualified ender
// before the next whitespace), evaluate its period context; for a cut, its realigned boundary.
template <bool kParams>
__device__ inline bool eval_candidate(const PunktTab& t, const Src& src, int64_t i, int64_t b0, int64_t b1,
                                      int64_t rs, int64_t* bound) {
  int64_t s2 = 0, e2 = 0, e1 = i + 1, next_start;
  if (non_word(src[i + 1])) {
    // finditer takes the LAST qualified ender of the run: any later one in the run wins
    for (int64_t k = i + 1; k < rs; ++k) {
      if (space_at(t, src, k, b0, b1)) break;
      if (sent_end(src[k]) && k + 1 < rs && (non_word(src[k + 1]) || space_at(t, src, k + 1, b0, b1)))
        return false;
    }
    e1 = i + 2;  // context = match + the NonWord char
    next_start = i + 1;
  } else {
    s2 = i + 1;
    while (space_at(t, src, s2, b0, b1)) ++s2;  // non-whitespace exists before rs
    e2 = s2;
    while (e2 < b1 && !space_at(t, src, e2, b0, b1)) ++e2;
    next_start = s2;
  }
  int64_t run_start = i;  // the match starts at the run's first byte
  while (run_start > b0 && !space_at(t, src, run_start - 1, b0, b1)) --run_start;
  if (!contains_sentbreak(t, src, run_start, e1, s2, e2)) return false;
  // _realign_boundaries: a closing run followed by whitespace, "--" or the end moves left
  int64_t k = next_start;
  while (k < rs && closing(src[k])) ++k;
  const bool ok = k > next_start &&
                  (k >= rs || space_at(t, src, k, b0, b1) || (src[k] == '-' && k + 1 < b1 && src[k + 1] == '-'));
  *bound = ok ? k : next_start;
  return true;
}

// K1: one wavefront per document streams it through a 4-KB LDS slab (four 16-B loads per lane
// in flight), 4 bytes per lane per 256-byte window, and appends each whitespace-free run's match
// -- its last lookahead-qualified sentence ender (text[q] in .?! and text[q+1] NonWord, or
// whitespace with non-whitespace later) -- in order to the document's slot range
// cand[(doc_off[d] - doc_off[0]) / 2 + d ..] (a document of L bytes has at most L/2 + 1
// whitespace-free runs, the bound of both candidates and cuts: "?!?!?! x" has five qualified
// enders in one run, so one per run is what keeps writes inside the range).
// 6 waves per SIMD (<= 80 VGPRs): 5.8 ms per 2 GiB vs 6.1 at the compiler's 96 VGPRs / 5 waves
// and 6.3 at 8 waves (64 VGPRs, spills) -- profiles/r01_v14_segment_variants.txt
__global__ void __launch_bounds__(64 * kSegWaves) __attribute__((amdgpu_waves_per_eu(6))) segment_classify_kernel(
    PunktTab t, const uint8_t* __restrict__ x, int64_t n_bytes, const int64_t* __restrict__ doc_off,
    int64_t n_doc, int32_t* __restrict__ cand, int32_t* __restrict__ ccnt, int32_t* __restrict__ rs_rel,
    int32_t* __restrict__ cnt) {
  __shared__ uint4 slab_all[kSegWaves][kSlab / 16];
  const int64_t d = (int64_t)blockIdx.x * kSegWaves + wave_id();
  if (d >= n_doc) return;  // wave-uniform
  const int lane = lane_id();
  uint4* slab = slab_all[threadIdx.x >> 6];
  const int64_t b0 = doc_off[d], b1 = doc_off[d + 1];
  int32_t* out = cand + ((b0 - doc_off[0]) >> 1) + d;
  const Src g(x, slab, 0, 0);  // global only
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
  int32_t nc = 0;
  for (int64_t blk = b0; blk < rs;) {
    const int64_t lo = blk & ~(int64_t)15;
    const int64_t hi = std::min<int64_t>(n_bytes, lo + kSlab);
    wave_sync();  // previous slab consumed
    if (aligned && lo + kSlab <= n_bytes) {  // all loads in flight before the LDS writes
      uint4 v[kSlab / 1024];
#pragma unroll
      for (int r = 0; r < kSlab / 1024; ++r)
        v[r] = *reinterpret_cast<const uint4*>(x + lo + 16 * (int64_t)(lane + 64 * r));
#pragma unroll
      for (int r = 0; r < kSlab / 1024; ++r) slab[lane + 64 * r] = v[r];
    } else {  // end of the text buffer / unaligned text: byte loads
      for (int r = lane; r < kSlab / 16; r += 64) {
        const int64_t a = lo + 16 * (int64_t)r;
        uint8_t tmp[16] = {};
        for (int k = 0; k < 16 && a + k < hi; ++k) tmp[k] = x[a + k];
        uint4 v;
        memcpy(&v, tmp, 16);
        slab[r] = v;
      }
    }
    wave_sync();
    const Src src(x, slab, lo, hi);
    const int64_t bend = std::min<int64_t>(rs, hi);
    const uint32_t* slab32 = reinterpret_cast<const uint32_t*>(slab);
    // 256-byte windows, 4 bytes per lane (one LDS dword); a SWAR test skips words without
    // '.', '?' or '!' (bytes before b0 -- first slab only -- are masked)
    for (int64_t base = lo; base < bend; base += 256) {
      const int64_t i0 = base + 4 * lane;
      const uint32_t w = slab32[(i0 - lo) >> 2];
      const uint32_t x1 = w ^ 0x2E2E2E2Eu, x2 = w ^ 0x3F3F3F3Fu, x3 = w ^ 0x21212121u;
      const uint32_t maybe = ((x1 - 0x01010101u) & ~x1) | ((x2 - 0x01010101u) & ~x2) |
                             ((x3 - 0x01010101u) & ~x3);
      uint32_t qb = 0, nwb = 0;
      if (maybe & 0x80808080u) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int64_t pos = i0 + k;
          const uint32_t c = (w >> (8 * k)) & 255u;
          if (pos < b0 || pos >= bend || !sent_end(c) || pos + 1 >= rs) continue;
          const uint32_t cn = k < 3 ? (w >> (8 * k + 8)) & 255u : src[pos + 1];
          if (non_word(cn))
            nwb |= 1u << k;
          else if (cn < 0x80 ? ascii_space(cn) : space_at(t, src, pos + 1, b0, b1))
            qb |= 1u << k;
        }
      }
      // a NonWord lookahead is a match only if it is the run's LAST qualified ender (finditer):
      // scan the rest of the run (rare; kept out of the unrolled loop above so its registers do
      // not cost occupancy). This also keeps the candidates within the per-document slot range.
      for (uint32_t m = nwb; m; m &= m - 1) {
        const int64_t pos = i0 + __builtin_ctz(m);
        bool last = true;
        for (int64_t q = pos + 1; q < rs && last; ++q) {
          if (space_at(t, src, q, b0, b1)) break;
          if (sent_end(src[q]) && q + 1 < rs && (non_word(src[q + 1]) || space_at(t, src, q + 1, b0, b1)))
            last = false;
        }
        if (last) qb |= m & (~m + 1);
      }
      if (ballot(qb != 0)) {  // append this window's enders in position order
        const int n = __builtin_popcount(qb);
        const int incl = wave_incl_scan(n);
        int slot = nc + incl - n;
        for (uint32_t m = qb; m; m &= m - 1) out[slot++] = (int32_t)(i0 + __builtin_ctz(m) - b0);
        nc += __shfl(incl, 63, 64);
      }
    }
    blk = bend;
  }
  if (lane == 0) {
    ccnt[d] = nc;
    rs_rel[d] = (int32_t)(rs - b0);
    cnt[d] = 1;
  }
}

struct CntAt {
  const int32_t* cnt;
  __device__ int64_t operator()(int64_t i) const { return cnt[i]; }
};

// K1b: candidates into one flat list (position, document), in document order
__global__ void segment_flatten_kernel(const int64_t* __restrict__ doc_off, int64_t n_doc,
                                       const int32_t* __restrict__ cand, const int64_t* __restrict__ coff,
                                       int64_t* __restrict__ fq, int32_t* __restrict__ fdoc) {
  const int64_t d = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave_id();
  if (d >= n_doc) return;
  const int64_t b0 = doc_off[d];
  const int32_t* in = cand + ((b0 - doc_off[0]) >> 1) + d;
  const int64_t o = coff[d], n = coff[d + 1] - o;
  for (int64_t k = lane_id(); k < n; k += 64) {
    fq[o + k] = b0 + in[k];
    fdoc[o + k] = (int32_t)d;
  }
}

// K2: one lane per candidate. The lane stages 64 bytes around its ender in a private LDS row
// (four 16-B loads issued together), then walks the context from LDS (Src falls back to global
// memory outside the row). fbound = realigned cut position, or -1; cnt[d] counts the cuts.
template <bool kParams>
__global__ void __launch_bounds__(kEvalBlock) segment_eval_kernel(
    PunktTab t, const uint8_t* __restrict__ x, int64_t n_bytes, const int64_t* __restrict__ doc_off,
    const int32_t* __restrict__ rs_rel, const int64_t* __restrict__ fq, const int32_t* __restrict__ fdoc,
    int64_t n_cand, int64_t* __restrict__ fbound, int32_t* __restrict__ cnt) {
  __shared__ uint32_t rows[kEvalBlock * kRowW];
  if (!kParams) t.n_rec = 0;
  const int64_t c = (int64_t)blockIdx.x * kEvalBlock + threadIdx.x;
  if (c >= n_cand) return;
  uint32_t* row = rows + threadIdx.x * kRowW;
  const int64_t q = fq[c];
  const int32_t d = fdoc[c];
  const int64_t b0 = doc_off[d], b1 = doc_off[d + 1], rs = b0 + rs_rel[d];
  const int64_t w0 = std::max<int64_t>(0, (q - 24) & ~(int64_t)15);
  const int64_t w1 = std::min<int64_t>(n_bytes, w0 + kCtx);
  uint4 v[kCtx / 16];
  const bool aligned = ((uintptr_t)x & 15u) == 0;
#pragma unroll
  for (int k = 0; k < kCtx / 16; ++k) {
    const int64_t a = w0 + 16 * k;
    v[k] = make_uint4(0, 0, 0, 0);
    if (a + 16 <= w1 && aligned) {
      v[k] = *reinterpret_cast<const uint4*>(x + a);
    } else if (a < w1) {
      uint8_t tmp[16] = {};
      for (int j = 0; j < 16 && a + j < w1; ++j) tmp[j] = x[a + j];
      memcpy(&v[k], tmp, 16);
    }
  }
#pragma unroll
  for (int k = 0; k < kCtx / 16; ++k) {
    row[4 * k] = v[k].x;
    row[4 * k + 1] = v[k].y;
    row[4 * k + 2] = v[k].z;
    row[4 * k + 3] = v[k].w;
  }
  const Src src(x, row, w0, w1);
  int64_t bound = -1;
  const bool cut = eval_candidate<kParams>(t, src, q, b0, b1, rs, &bound);
  fbound[c] = cut ? bound : -1;
  if (cut) atomicAdd(&cnt[d], 1);
}

// sent_off[doc_sent_off[d] + k]: document start, then its cuts in order; sent_off[n_sent] = end
__global__ void segment_fill_kernel(const int64_t* __restrict__ doc_off, int64_t n_doc,
                                    const int64_t* __restrict__ coff, const int64_t* __restrict__ fbound,
                                    const int64_t* __restrict__ dso, int64_t* __restrict__ sent_off) {
  const int64_t d = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave_id();
  if (d >= n_doc) return;
  const int lane = lane_id();
  const int64_t o = dso[d];
  if (lane == 0) sent_off[o] = doc_off[d];
  int64_t k = o + 1;
  for (int64_t base = coff[d], e = coff[d + 1]; base < e; base += 64) {
    const int64_t j = base + lane;
    const int64_t bnd = j < e ? fbound[j] : -1;
    const uint64_t m = ballot(bnd >= 0);
    if (bnd >= 0) sent_off[k + popc_below(m)] = bnd;
    k += __builtin_popcountll(m);
  }
  if (d == n_doc - 1 && lane == 0) sent_off[dso[n_doc]] = doc_off[n_doc];
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
  DevArena::Block cand, ccnt, rs_rel, coff, fq, fdoc, fbound, cnt, dso, scratch;
  const int64_t* doc_off = nullptr;
  int64_t n_doc = -1;
  int64_t n_sent = 0;
  std::vector<DevArena::Block*> blocks() {
    return {&cand, &ccnt, &rs_rel, &coff, &fq, &fdoc, &fbound, &cnt, &dso, &scratch};
  }
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
  for (DevArena::Block* b : p->blocks())
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
  DevArena& A = c->arena;
  const size_t nd = (size_t)n_doc + 1;
  LDDL_HIP(A.take(sizeof(int32_t) * (size_t)(n_bytes / 2 + n_doc + 2), st, ps->cand));
  LDDL_HIP(A.take(sizeof(int32_t) * nd, st, ps->ccnt));
  LDDL_HIP(A.take(sizeof(int32_t) * nd, st, ps->rs_rel));
  LDDL_HIP(A.take(sizeof(int32_t) * nd, st, ps->cnt));
  LDDL_HIP(A.take(sizeof(int64_t) * nd, st, ps->coff));
  LDDL_HIP(A.take(sizeof(int64_t) * nd, st, ps->dso));
  LDDL_HIP(A.take(sizeof(int64_t) * (size_t)scan_scratch_elems(n_doc), st, ps->scratch));
  PunktTab t{ps->l1, ps->pages, ps->lower, ps->n_lower, ps->hash, ps->hmask, ps->n_rec, ps->keys};
  int32_t* ccnt = static_cast<int32_t*>(ps->ccnt.p);
  int32_t* cnt = static_cast<int32_t*>(ps->cnt.p);
  int64_t* coff = static_cast<int64_t*>(ps->coff.p);
  int64_t* dso = static_cast<int64_t*>(ps->dso.p);
  int64_t* scratch = static_cast<int64_t*>(ps->scratch.p);
  const int64_t dgrid = std::max<int64_t>(1, (n_doc + kSegWaves - 1) / kSegWaves);
  if (n_doc > 0) {
    hipLaunchKernelGGL(segment_classify_kernel, dim3((unsigned)dgrid), dim3(64 * kSegWaves), 0, st, t, d_text,
                       n_bytes, d_doc_off, n_doc, static_cast<int32_t*>(ps->cand.p), ccnt,
                       static_cast<int32_t*>(ps->rs_rel.p), cnt);
    LDDL_HIP(hipGetLastError());
  }
  LDDL_HIP(scan_exclusive(CntAt{ccnt}, n_doc, coff, scratch, st));
  int64_t n_cand = 0;
  LDDL_HIP(hipMemcpyAsync(&n_cand, coff + n_doc, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  LDDL_HIP(hipStreamSynchronize(st));
  const size_t ncap = (size_t)std::max<int64_t>(n_cand, 1);
  LDDL_HIP(A.take(sizeof(int64_t) * ncap, st, ps->fq));
  LDDL_HIP(A.take(sizeof(int32_t) * ncap, st, ps->fdoc));
  LDDL_HIP(A.take(sizeof(int64_t) * ncap, st, ps->fbound));
  if (n_cand > 0) {
    hipLaunchKernelGGL(segment_flatten_kernel, dim3((unsigned)dgrid), dim3(64 * kSegWaves), 0, st, d_doc_off,
                       n_doc, static_cast<const int32_t*>(ps->cand.p), coff, static_cast<int64_t*>(ps->fq.p),
                       static_cast<int32_t*>(ps->fdoc.p));
    const int64_t egrid = (n_cand + kEvalBlock - 1) / kEvalBlock;
    if (ps->n_rec)
      hipLaunchKernelGGL(segment_eval_kernel<true>, dim3((unsigned)egrid), dim3(kEvalBlock), 0, st, t, d_text,
                         n_bytes, d_doc_off, static_cast<const int32_t*>(ps->rs_rel.p),
                         static_cast<const int64_t*>(ps->fq.p), static_cast<const int32_t*>(ps->fdoc.p), n_cand,
                         static_cast<int64_t*>(ps->fbound.p), cnt);
    else
      hipLaunchKernelGGL(segment_eval_kernel<false>, dim3((unsigned)egrid), dim3(kEvalBlock), 0, st, t, d_text,
                         n_bytes, d_doc_off, static_cast<const int32_t*>(ps->rs_rel.p),
                         static_cast<const int64_t*>(ps->fq.p), static_cast<const int32_t*>(ps->fdoc.p), n_cand,
                         static_cast<int64_t*>(ps->fbound.p), cnt);
    LDDL_HIP(hipGetLastError());
  }
  LDDL_HIP(scan_exclusive(CntAt{cnt}, n_doc, dso, scratch, st));
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
  if (!d_sent_off && !d_doc_sent_off) {  // cancel: release the pending segmentation's scratch
    for (DevArena::Block* b : ps->blocks()) {
      c->arena.give(*b, st);
      *b = DevArena::Block{};
    }
    ps->n_doc = -1;
    return 0;
  }
  if (!d_sent_off || !d_doc_sent_off) LDDL_FAIL(-1, "lddl_segment_fill: null output");
  const int64_t n_doc = ps->n_doc;
  int rc = 0;
  if (n_doc > 0) {
    const int64_t grid = (n_doc + 3) / 4;
    hipLaunchKernelGGL(segment_fill_kernel, dim3((unsigned)grid), dim3(256), 0, st, ps->doc_off, n_doc,
                       static_cast<const int64_t*>(ps->coff.p), static_cast<const int64_t*>(ps->fbound.p),
                       static_cast<const int64_t*>(ps->dso.p), d_sent_off);
  } else {
    if (hipMemsetAsync(d_sent_off, 0, sizeof(int64_t), st) != hipSuccess) rc = -100;
  }
  if (hipMemcpyAsync(d_doc_sent_off, ps->dso.p, sizeof(int64_t) * (size_t)(n_doc + 1), hipMemcpyDeviceToDevice,
                     st) != hipSuccess)
    rc = -100;
  if (hipGetLastError() != hipSuccess) rc = -100;
  for (DevArena::Block* b : ps->blocks()) {
    c->arena.give(*b, st);
    *b = DevArena::Block{};
  }
  ps->n_doc = -1;
  if (rc) LDDL_FAIL(rc, "lddl_segment_fill: HIP launch/copy failed");
  return 0;
}
