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
    int64_t n_sent, int32_t max_pieces, int32_t* __restrict__ ids, int32_t* __restrict__ sent_len) {
  __shared__ uint8_t wbuf_all[kBlock * kWordStride];
  const int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (s >= n_sent) return;
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

}  // namespace
}  // namespace lddl

using namespace lddl;

extern "C" int lddl_tokenize(lddl_ctx* c, void* stream, const uint8_t* d_text, int64_t n_bytes,
                             const int64_t* d_sent_off, int64_t n_sent, int32_t max_pieces,
                             int32_t* d_ids, int32_t* d_sent_len) {
  if (!c) LDDL_FAIL(-1, "null ctx");
  if (n_sent < 0 || n_bytes < 0 || max_pieces <= 0) LDDL_FAIL(-1, "bad sizes");
  if (n_sent == 0) return 0;
  const int64_t grid = (n_sent + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(tokenize_lane_kernel, dim3((unsigned)grid), dim3(kBlock), 0, as_stream(stream),
                     c->tab, d_text, d_sent_off, n_sent, max_pieces, d_ids, d_sent_len);
  LDDL_HIP(hipGetLastError());
  return 0;
}
