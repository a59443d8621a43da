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
// Two kernels:
//   tokenize_wave_kernel   one wavefront per sentence (grid-stride). The sentence is consumed in
//                          64-byte windows, one byte per lane (coalesced loads). Lanes classify
//                          their code point (ASCII via an LDS copy of the table page, UTF-8 leads
//                          decoded in place), ballots find the pre-tokenizer units (word runs,
//                          isolated chars, literal special tokens), then lane k runs greedy
//                          longest-match WordPiece on unit k: ASCII words of <= 16 bytes with the
//                          word held in two 64-bit registers (SWAR lowercase, hash keys by shift
//                          and mask), everything else from a per-lane LDS buffer. A wave prefix
//                          scan of the per-unit piece counts places the pieces. A unit that does
//                          not fit a window, a word of > kPcs pieces or a normalised word of
//                          > kNorm bytes sends the whole sentence to the fallback list.
//   tokenize_lane_kernel   one lane per listed sentence, sequential (unbounded words, 100-char
//                          rule); also the whole-corpus path when LDDL_TOKENIZE_PATH=lane.
#include <algorithm>
#include <cstdlib>
#include <cstring>

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
constexpr int kNorm = 48;  // normalised bytes per unit on the generic path (more -> fallback)

// unit categories per byte position
enum : uint32_t { kCatRun = 0, kCatSep = 1, kCatIso = 2, kCatSpecial = 3 };

struct alignas(16) WaveLds {
  uint8_t win[64 + 16];        // window bytes (+16 so 20-byte reads at any start stay inside)
  uint8_t us[64], ue[64], uk[64];  // unit k: first byte, last byte (window-relative), kind
  int32_t pcs[kPcs * 64];      // lane l's pieces at pcs[j * 64 + l]
  uint8_t nrm[64 * kNorm];     // lane l's normalised word (generic path)
};

// Order this wave's LDS writes before its later LDS reads of other lanes' data (the waves of a
// workgroup work on different sentences, so a workgroup barrier would not be uniform).
__device__ inline void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ inline uint64_t lanes_below() { return (1ull << lane_id()) - 1ull; }

__device__ inline int match_special_at(const Tables& T, const uint8_t* b, int64_t i, int64_t end) {
  for (int k = 0; k < kNumSpecial; ++k)
    if (T.special_id[k] >= 0 && match_special(b, i, end, k)) return k;
  return -1;
}

// 128-bit little-endian byte string shifted down by `sh` bytes (0..15)
__device__ inline void shr128(uint64_t lo, uint64_t hi, int sh, uint64_t& a, uint64_t& b) {
  if (sh == 0) { a = lo; b = hi; }
  else if (sh < 8) { a = (lo >> (8 * sh)) | (hi << (64 - 8 * sh)); b = hi >> (8 * sh); }
  else { a = hi >> (8 * (sh - 8)); b = 0; }
}

// Vocab probe for a key held in registers: bytes [0,8) in a, [8,16) in b (len <= 16).
__device__ inline int32_t probe_reg(const Tables& T, uint64_t a, uint64_t b, int len, uint32_t cont) {
  const uint64_t k0 = keep_bytes(a, len);
  const uint32_t k1 = (uint32_t)keep_bytes(b, len - 8 < 4 ? len - 8 : 4);
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
      for (int i = 12; i < len; ++i) ok &= p[i] == (uint8_t)(b >> (8 * (i - 8)));
      if (ok) return id;
    }
  }
}

// Greedy longest-match WordPiece of an ASCII word of nb <= 16 bytes held in (lo, hi).
// Returns the piece count written to pc[j * 64] (j < kPcs), or -1 if more than kPcs pieces.
__device__ int wordpiece_reg(const Tables& T, uint64_t lo, uint64_t hi, int nb, int32_t* pc) {
  int n = 0, start = 0;
  while (start < nb) {
    uint64_t a, b;
    shr128(lo, hi, start, a, b);
    int len = nb - start < T.max_piece_bytes ? nb - start : T.max_piece_bytes;
    int32_t id = -1;
    for (; len > 0; --len) {
      id = probe_reg(T, a, b, len, start > 0);
      if (id >= 0) break;
    }
    if (id < 0) {
      pc[0] = T.special_id[kUnk];
      return 1;
    }
    if (n == kPcs) return -1;
    pc[64 * n++] = id;
    start += len;
  }
  return n;
}

// Greedy longest-match WordPiece of a normalised word in LDS (UTF-8, nb bytes, nc chars).
__device__ int wordpiece_lds(const Tables& T, const uint8_t* w, int nb, int nc, int32_t* pc) {
  if (nc == 0) return 0;
  if (nc > 100) { pc[0] = T.special_id[kUnk]; return 1; }
  int n = 0, start = 0;
  while (start < nb) {
    int end = nb < start + T.max_piece_bytes ? nb : start + T.max_piece_bytes;
    int32_t found = -1;
    for (; end > start; --end) {
      if (end < nb && (w[end] & 0xC0) == 0x80) continue;  // not a char boundary
      found = lookup(T, w, start, end - start, start > 0);
      if (found >= 0) break;
    }
    if (found < 0) { pc[0] = T.special_id[kUnk]; return 1; }
    if (n == kPcs) return -1;
    pc[64 * n++] = found;
    start = end;
  }
  return n;
}

__global__ void __launch_bounds__(64 * kTW) tokenize_wave_kernel(
    Tables T, const uint8_t* __restrict__ text, const int64_t* __restrict__ sent_off,
    int64_t n_sent, int32_t max_pieces, int32_t* __restrict__ ids, int32_t* __restrict__ sent_len,
    int32_t* __restrict__ fb_list, uint32_t* __restrict__ fb_n) {
  __shared__ uint32_t s_ascii[128];
  __shared__ WaveLds s_w[kTW];
  for (int c = threadIdx.x; c < 128; c += blockDim.x) s_ascii[c] = tab_entry(T, (uint32_t)c);
  __syncthreads();
  const int lane = lane_id();
  WaveLds& W = s_w[threadIdx.x >> 6];
  const uint64_t below = lanes_below();
  const bool lower = T.ascii_mode == 1;
  const bool fast_ok = T.ascii_mode != 0;
  const int64_t stride = (int64_t)gridDim.x * kTW;
  for (int64_t s = (int64_t)blockIdx.x * kTW + (threadIdx.x >> 6); s < n_sent; s += stride) {
    const int64_t b0 = sent_off[s], b1 = sent_off[s + 1];
    int64_t pos = b0;
    int32_t emitted = 0, flags = 0;
    bool fallback = false;
    while (pos < b1 && emitted < max_pieces) {
      const int64_t i = pos + lane;
      const bool in = i < b1;
      const uint32_t byte = in ? text[i] : 0x20u;
      W.win[lane] = (uint8_t)byte;
      // ---- classify this lane's byte -----------------------------------------------------
      uint32_t cls = kSpace;  // beyond the sentence: a separator
      int cplen = 1;          // bytes of the code point starting here (0: covered continuation)
      int spk = -1;           // literal special token starting here
      bool slow = false;      // non-ASCII or dropped char: not for the register fast path
      bool cont = false;
      if (in) {
        if (byte < 0x80) {
          cls = s_ascii[byte] >> 30;
          slow = cls == kDrop;
          if (byte == '[') spk = match_special_at(T, text, i, b1);
        } else if (byte >= 0xC0) {
          int64_t j = i;
          const uint32_t cp = utf8_next(text, b1, j);
          cplen = (int)(j - i);
          cls = tab_entry(T, cp) >> 30;
          slow = true;
        } else {
          cont = true;  // resolved below: covered by a valid lead, or a lone byte (U+FFFD, drop)
          cls = kDrop;
          slow = true;
        }
      }
      const uint64_t V2 = __ballot(cplen == 2), V3 = __ballot(cplen == 3), V4 = __ballot(cplen == 4);
      const uint64_t C1 = (V2 | V3 | V4) << 1, C2 = (V3 | V4) << 2, C3 = V4 << 3;
      const bool covered = cont && (((C1 | C2 | C3) >> lane) & 1ull);
      const int dist = !covered ? 0 : ((C1 >> lane) & 1ull) ? 1 : ((C2 >> lane) & 1ull) ? 2 : 3;
      // a covered continuation inherits its lead's class; cp_last marks a code point's last byte
      const int lead_len = __shfl((int)(cls | ((uint32_t)cplen << 4)), lane - dist, 64);
      if (covered) {
        cls = (uint32_t)lead_len & 3u;
        cplen = 0;
      }
      const bool cp_last = covered ? (dist == (lead_len >> 4) - 1) : (cplen <= 1);
      const uint64_t S = __ballot(spk >= 0), S6 = __ballot(spk == kMask);
      const uint64_t inside = (S << 1) | (S << 2) | (S << 3) | (S << 4) | (S6 << 5);
      const bool in_sp = ((S | inside) >> lane) & 1ull;
      const uint32_t cat = in_sp ? kCatSpecial
                                 : cls == kSpace ? kCatSep : cls == kIso ? kCatIso : kCatRun;
      const uint64_t RUN = __ballot(cat == kCatRun);
      const uint64_t LEAD = __ballot(cplen > 0);
      const uint64_t ISO = __ballot(cat == kCatIso);
      const uint64_t CPL = __ballot(cp_last);
      const uint64_t SLOW = __ballot(slow);
      const bool tail_known = pos + 64 >= b1;  // position 64 is past the sentence end
      const uint64_t US = S | (ISO & LEAD) | (RUN & ~(RUN << 1));
      uint64_t RE = RUN & ~(RUN >> 1);
      if (!tail_known) RE &= ~(1ull << 63);
      const uint64_t UE = ((S & ~S6) << 4) | (S6 << 5) | (ISO & CPL & ~inside) | RE;
      const int n_units = __popcll(UE);
      const int n_starts = __popcll(US);
      int64_t next;
      if (n_starts > n_units) {
        const int last = 63 - __clzll(US);
        if (last == 0) { fallback = true; break; }  // a unit of >= 64 bytes
        next = pos + last;
      } else if (tail_known) {
        next = b1;
      } else {
        // a separator code point straddling the window end restarts the next window at its lead
        const int hl = 63 - __clzll(LEAD);
        const int hc = 63 - __clzll(CPL);
        next = pos + (hl > hc ? hl : 64);
      }
      if ((US >> lane) & 1ull) {
        const int k = __popcll(US & below);
        W.us[k] = (uint8_t)lane;
        W.uk[k] = (uint8_t)(spk >= 0 ? 2 + spk : cat == kCatIso ? 1 : 0);
      }
      if ((UE >> lane) & 1ull) W.ue[__popcll(UE & below)] = (uint8_t)lane;
      wave_sync();
      // ---- WordPiece: lane k takes unit k --------------------------------------------------
      int npc = 0;
      bool cs_flag = false;
      int32_t* pc = W.pcs + lane;
      if (lane < n_units) {
        const int us = W.us[lane], ue = W.ue[lane], kind = W.uk[lane];
        const int ulen = ue - us + 1;
        if (kind >= 2) {
          pc[0] = T.special_id[kind - 2];
          npc = 1;
          cs_flag = kind - 2 == kCls || kind - 2 == kSep;
        } else {
          const bool unit_slow = ((SLOW >> us) & (ulen >= 64 ? ~0ull : ((1ull << ulen) - 1))) != 0;
          if (kind == 0 && !unit_slow && ulen <= 16 && fast_ok) {
            const uint32_t* wd = reinterpret_cast<const uint32_t*>(W.win) + (us >> 2);
            const int r = us & 3;
            const uint32_t d0 = wd[0], d1 = wd[1], d2 = wd[2], d3 = wd[3], d4 = wd[4];
            const uint32_t a0 = __builtin_amdgcn_alignbyte(d1, d0, r);
            const uint32_t a1 = __builtin_amdgcn_alignbyte(d2, d1, r);
            const uint32_t a2 = __builtin_amdgcn_alignbyte(d3, d2, r);
            const uint32_t a3 = __builtin_amdgcn_alignbyte(d4, d3, r);
            uint64_t lo = keep_bytes((uint64_t)a0 | ((uint64_t)a1 << 32), ulen);
            uint64_t hi = keep_bytes((uint64_t)a2 | ((uint64_t)a3 << 32), ulen - 8);
            if (lower) {  // SWAR A-Z -> a-z on ASCII bytes
              const uint64_t k3f = 0x3f3f3f3f3f3f3f3full, k25 = 0x2525252525252525ull,
                             k80 = 0x8080808080808080ull;
              lo |= (((lo + k3f) & ~(lo + k25)) & k80) >> 2;
              hi |= (((hi + k3f) & ~(hi + k25)) & k80) >> 2;
            }
            npc = wordpiece_reg(T, lo, hi, ulen, pc);
          } else {
            // generic: normalise the unit's code points into the lane's LDS buffer
            uint8_t* w = W.nrm + lane * kNorm;
            int nb = 0, nc = 0;
            int64_t j = pos + us;
            const int64_t je = pos + ue + 1;
            while (j < je && nb >= 0) {
              const uint32_t cp = utf8_next(text, b1, j);
              const uint32_t e = tab_entry(T, cp);
              if ((e >> 30) == kDrop) continue;
              uint8_t ob[12];
              int olen, ochars = 1;
              if (e & kIdent) olen = put_utf8(ob, cp);
              else if (e & kMulti) {
                const uint8_t* p = T.pool + (e & 0xFFFFFFu);
                olen = p[0];
                ochars = p[1];
                for (int q = 0; q < olen; ++q) ob[q] = p[2 + q];
              } else olen = put_utf8(ob, e & 0x1FFFFFu);
              if (nb + olen > kNorm) { nb = -1; break; }
              for (int q = 0; q < olen; ++q) w[nb + q] = ob[q];
              nb += olen;
              nc += ochars;
            }
            npc = nb < 0 ? -1 : wordpiece_lds(T, w, nb, nc, pc);
          }
        }
      }
      if (__ballot(npc < 0)) { fallback = true; break; }
      // ---- place the pieces ----------------------------------------------------------------
      const int incl = wave_incl_scan(npc);
      const int excl = incl - npc;
      const int total = __shfl(incl, 63, 64);
      const int o = emitted + excl;
      for (int q = 0; q < npc; ++q)
        if (o + q < max_pieces) ids[b0 + o + q] = pc[64 * q];
      if (__ballot(cs_flag && o < max_pieces)) flags = kLenHasClsSep;
      emitted += total;
      pos = next;
      wave_sync();
    }
    if (fallback) {
      if (lane == 0) fb_list[atomicAdd(fb_n, 1u)] = (int32_t)s;
    } else if (lane == 0) {
      sent_len[s] = (emitted < max_pieces ? emitted : max_pieces) | flags;
    }
  }
}

}  // namespace
}  // namespace lddl

using namespace lddl;

extern "C" int lddl_tokenize(lddl_ctx* c, void* stream, const uint8_t* d_text, int64_t n_bytes,
                             const int64_t* d_sent_off, int64_t n_sent, int32_t max_pieces,
                             int32_t* d_ids, int32_t* d_sent_len) {
  if (!c) LDDL_FAIL(-1, "null ctx");
  if (n_sent < 0 || n_bytes < 0 || max_pieces <= 0) LDDL_FAIL(-1, "bad sizes");
  if (n_sent >= (int64_t)INT32_MAX) LDDL_FAIL(-1, "too many sentences in one call (%lld)", (long long)n_sent);
  if (n_sent == 0) return 0;
  hipStream_t st = as_stream(stream);
  const char* path = getenv("LDDL_TOKENIZE_PATH");  // diagnostics: "lane" = fallback kernel only
  if (path && !strcmp(path, "lane")) {
    const int64_t grid = std::min<int64_t>((n_sent + kBlock - 1) / kBlock, 65536);
    hipLaunchKernelGGL(tokenize_lane_kernel, dim3((unsigned)grid), dim3(kBlock), 0, st, c->tab,
                       d_text, d_sent_off, n_sent, max_pieces, d_ids, d_sent_len, nullptr, nullptr);
    LDDL_HIP(hipGetLastError());
    return 0;
  }
  // fallback list: [0] = count, then sentence indices
  int32_t* fb;
  LDDL_HIP(hipMallocAsync((void**)&fb, sizeof(int32_t) * (size_t)(n_sent + 1), st));
  LDDL_HIP(hipMemsetAsync(fb, 0, sizeof(int32_t), st));
  int n_cu = 256;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, c->device);
  // grid-stride over sentences with exactly the resident workgroups (a second wave of
  // workgroups would start only when the first finished: a 2x tail)
  int per_cu = 0;
  LDDL_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, tokenize_wave_kernel, 64 * kTW, 0));
  const int64_t want = (n_sent + kTW - 1) / kTW;
  const int64_t grid = std::min<int64_t>(want, (int64_t)n_cu * std::max(per_cu, 1));
  hipLaunchKernelGGL(tokenize_wave_kernel, dim3((unsigned)grid), dim3(64 * kTW), 0, st, c->tab,
                     d_text, d_sent_off, n_sent, max_pieces, d_ids, d_sent_len, fb + 1,
                     reinterpret_cast<uint32_t*>(fb));
  const int64_t fgrid = std::min<int64_t>((n_sent + kBlock - 1) / kBlock, (int64_t)n_cu * 2);
  hipLaunchKernelGGL(tokenize_lane_kernel, dim3((unsigned)fgrid), dim3(kBlock), 0, st, c->tab,
                     d_text, d_sent_off, n_sent, max_pieces, d_ids, d_sent_len, fb + 1,
                     reinterpret_cast<const uint32_t*>(fb));
  LDDL_HIP(hipGetLastError());
  LDDL_HIP(hipFreeAsync(fb, st));
  return 0;
}
