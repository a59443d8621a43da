// Loader-side collate + dynamic masking (lddl/torch/bert.py:69-196) on the GPU.
//
//   lddl_collate_encode   _to_encoded_inputs (bert.py:69-149): whitespace-split the A / B strings
//                         of a batch, convert_tokens_to_ids (exact vocab lookup, [UNK] if absent),
//                         fill input_ids / token_type_ids / attention_mask and either
//                         special_tokens_mask (dynamic) or labels from masked_lm_positions /
//                         masked_lm_labels (static). One wave per sample.
//   lddl_mask_dynamic     _mask_tokens (bert.py:152-196): per slot masked ~ Bernoulli(p) unless
//                         special; of the masked, Bernoulli(0.8) -> [MASK], else Bernoulli(0.5) ->
//                         random id in [0, len(tokenizer)), else unchanged; labels = id where
//                         masked, ignore_index elsewhere. Native mode draws from a counter-based
//                         Philox4x32-10 keyed by (seed, counter, slot); replay mode applies
//                         captured torch masks bit for bit.
//   lddl_collate_encode_masked   _to_encoded_inputs + _mask_tokens in ONE pass (the loader's
//                         dynamic-masking collate, bert.py:348-365): the row is built in LDS and
//                         masked on its way out, so input_ids / token_type_ids / attention_mask /
//                         labels are each written once (36 B per slot incl. the string read)
//                         and no special_tokens_mask is materialised; bit-identical to
//                         lddl_collate_encode followed by lddl_mask_dynamic (same Philox stream).
#include "common.h"
#include "ctx.h"
#include "device.h"
#include "lddl_amd.h"

namespace lddl {
namespace {

__device__ inline float u01(uint32_t x) { return (x >> 8) * (1.0f / 16777216.0f); }

// exact token string -> id (convert_tokens_to_ids); "##x" is the continuation entry of "x"
__device__ int32_t token_lookup(const Tables& T, const uint8_t* s, int len) {
  uint32_t cont = 0;
  if (len > 2 && s[0] == '#' && s[1] == '#') { cont = 1; s += 2; len -= 2; }
  if (len > 255) return -1;
  uint64_t k0 = 0;
  uint32_t k1 = 0;
  for (int i = 0; i < len && i < 8; ++i) k0 |= (uint64_t)s[i] << (8 * i);
  for (int i = 8; i < len && i < 12; ++i) k1 |= (uint32_t)s[i] << (8 * (i - 8));
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
      for (int i = 12; i < len; ++i) ok &= p[i] == s[i];
      if (ok) return id;
    }
  }
}

__device__ inline bool is_ws(uint8_t c) { return c == ' ' || (c >= 9 && c <= 13); }

// Split bytes[b0,b1) on whitespace and look every token up; token t -> out[t] (t < max_tok).
// Whole wave cooperates: 64-byte windows, word starts found by ballot. Returns #tokens.
__device__ int32_t split_lookup(const Tables& T, const uint8_t* bytes, int64_t b0, int64_t b1,
                                int32_t* out, int32_t max_tok, const uint16_t* scatter,
                                int32_t limit) {
  const int lane = lane_id();
  int32_t ntok = 0;
  uint8_t prev = ' ';
  for (int64_t base = b0; base < b1; base += 64) {
    const int64_t i = base + lane;
    const uint8_t c = i < b1 ? bytes[i] : ' ';
    const int up = __shfl_up((int)c, 1, 64);  // every lane must take part in the shuffle
    const uint8_t pc = lane == 0 ? prev : (uint8_t)up;
    const bool start = !is_ws(c) && is_ws(pc);
    const uint64_t m = __ballot(start);
    if (start) {
      const int32_t t = ntok + __popcll(m & ((1ull << lane) - 1));
      int64_t e = i;
      while (e < b1 && !is_ws(bytes[e])) ++e;
      int32_t id = token_lookup(T, bytes + i, (int)(e - i));
      if (id < 0) id = T.special_id[kUnk];
      if (t < max_tok) {
        const int32_t dst = scatter ? (int32_t)scatter[t] : t;
        if (dst < limit) out[dst] = id;  // a masked position >= L is refused on the host
      }
    }
    ntok += __popcll(m);
    prev = (uint8_t)__shfl((int)c, 63, 64);
  }
  return ntok;
}

// One slot's native-RNG masking decision (bert.py:176-192): Philox4x32-10 keyed by seed, counter
// (batch) and the flat slot index. Returns the output id; *label = id if masked else ignore.
struct MaskDraw {
  float p;
  int64_t ignore_index, mask_id, vocab_len;
  uint64_t seed, counter;
};
__device__ inline int64_t mask_slot(const MaskDraw& D, int64_t flat, bool special, int64_t id,
                                    int64_t* label) {
  const uint4 r = Philox::gen(make_uint4((uint32_t)flat, (uint32_t)(flat >> 32), (uint32_t)D.counter,
                                         (uint32_t)(D.counter >> 32)),
                              make_uint2((uint32_t)D.seed, (uint32_t)(D.seed >> 32)));
  const bool masked = !special && u01(r.x) < D.p;
  const bool replaced = masked && u01(r.y) < 0.8f;
  const bool rnd = masked && !replaced && u01(r.z) < 0.5f;
  *label = masked ? id : D.ignore_index;
  if (replaced) return D.mask_id;
  if (rnd) return (int64_t)(((uint64_t)r.w * (uint64_t)D.vocab_len) >> 32);
  return id;
}

struct EncodeArgs {
  Tables T;
  const uint8_t* bytes;
  const int64_t* a_off;  // [B+1] A string of sample b = bytes[a_off[b], a_off[b+1])
  const int64_t* b_off;  // [B+1]
  const int32_t* na;     // [B] token counts of A / B (host-computed, they size the batch)
  const int32_t* nb;
  int32_t B, L;
  int64_t* input_ids;
  int64_t* token_type_ids;
  int64_t* attention_mask;
  int64_t* special_tokens_mask;  // dynamic masking (nullable)
  // static masking (all nullable)
  const uint8_t* lab_bytes;
  const int64_t* lab_off;
  const uint16_t* pos;
  const int64_t* pos_off;
  int64_t* labels;
  int64_t ignore_index;
  int32_t fused_mask;  // 1: dynamic masking applied on the way out (labels written from it)
  MaskDraw draw;
};

constexpr int kEncWaves = 4;

// One wave per sample; the row is staged in LDS (ids, labels as int32) in two barrier-separated
// phases so that every output element is written exactly once, coalesced.
__global__ void __launch_bounds__(64 * kEncWaves) encode_kernel(EncodeArgs E) {
  extern __shared__ __attribute__((aligned(16))) int32_t srow[];
  const int w = wave_id(), lane = threadIdx.x & 63;
  const int b = blockIdx.x * kEncWaves + w;
  const bool active = b < E.B;
  int32_t* sid = srow + (size_t)w * 2 * E.L;
  int32_t* slab = sid + E.L;
  const int32_t na = active ? E.na[b] : 0, nb = active ? E.nb[b] : 0;
  const int32_t end = na + nb + 3;
  const int32_t cls = E.T.special_id[kCls], sep = E.T.special_id[kSep];
  if (active) {
    for (int32_t x = lane; x < E.L; x += 64) {
      if (x == 0) sid[x] = cls;
      else if (x == na + 1 || x == end - 1) sid[x] = sep;
      else if (x >= end) sid[x] = 0;
      slab[x] = -1;
    }
  }
  __syncthreads();
  if (active) {
    split_lookup(E.T, E.bytes, E.a_off[b], E.a_off[b + 1], sid + 1, na, nullptr, E.L);
    split_lookup(E.T, E.bytes, E.b_off[b], E.b_off[b + 1], sid + na + 2, nb, nullptr, E.L);
    if (E.labels && E.lab_bytes) {  // labels[b, positions] = ids of masked_lm_labels (bert.py:120-125)
      const int64_t p0 = E.pos_off[b];
      split_lookup(E.T, E.lab_bytes, E.lab_off[b], E.lab_off[b + 1], slab,
                   (int32_t)(E.pos_off[b + 1] - p0), E.pos + p0, E.L);
    }
  }
  __syncthreads();
  if (!active) return;
  const int64_t row = (int64_t)b * E.L;
  for (int32_t x = lane; x < E.L; x += 64) {
    const bool special = x == 0 || x == na + 1 || x >= end - 1;
    if (E.fused_mask) {
      int64_t lab;
      E.input_ids[row + x] = mask_slot(E.draw, row + x, special, sid[x], &lab);
      E.labels[row + x] = lab;
    } else {
      E.input_ids[row + x] = sid[x];
      if (E.labels) E.labels[row + x] = slab[x] < 0 ? E.ignore_index : (int64_t)slab[x];
    }
    E.token_type_ids[row + x] = (x >= na + 2 && x < end) ? 1 : 0;
    E.attention_mask[row + x] = x < end ? 1 : 0;
    if (E.special_tokens_mask) E.special_tokens_mask[row + x] = special ? 1 : 0;
  }
}

struct MaskArgs {
  int64_t* ids;        // [B, L] in/out
  int64_t* labels;     // [B, L] out
  const int64_t* special;  // [B, L] special_tokens_mask (nullable -> derived from na/nb, or
                           // without lengths from the ids: get_special_tokens_mask)
  const int32_t* na;
  const int32_t* nb;
  int64_t B, L;
  float p;
  int64_t ignore_index, mask_id, vocab_len;
  int32_t special_ids[kNumSpecial];  // [PAD] [UNK] [CLS] [SEP] [MASK] (-1 if absent)
  uint64_t seed, counter;
  // replay (all or none)
  const uint8_t* r_masked;
  const uint8_t* r_replaced;
  const uint8_t* r_random;
  const int64_t* r_words;
};

// special_tokens_mask of slot i = (b, x): the given tensor, else the layout from the lengths,
// else membership of the id in the special ids
__device__ inline bool mask_special(const MaskArgs& M, int64_t i, int64_t b, int64_t x, int64_t id) {
  if (M.special) return M.special[i] != 0;
  if (M.na) {
    const int32_t na = M.na[b], end = na + M.nb[b] + 3;
    return x == 0 || x == na + 1 || x >= end - 1;
  }
  bool sp = false;  // tokenizer.get_special_tokens_mask(ids, already_has_special_tokens=True)
  for (int k = 0; k < kNumSpecial; ++k) sp |= M.special_ids[k] >= 0 && id == M.special_ids[k];
  return sp;
}

__global__ void __launch_bounds__(256) mask_kernel(MaskArgs M) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= M.B * M.L) return;
  const int64_t b = i / M.L, x = i - b * M.L;
  const int64_t id = M.ids[i];
  const bool special = mask_special(M, i, b, x, id);
  if (!M.r_masked) {  // native: the shared Philox decision (also used by the fused collate)
    int64_t lab;
    const int64_t out = mask_slot(MaskDraw{M.p, M.ignore_index, M.mask_id, M.vocab_len, M.seed,
                                           M.counter}, i, special, id, &lab);
    M.labels[i] = lab;
    if (out != id) M.ids[i] = out;
    return;
  }
  // replay of captured torch draws: masked_indices already excludes special slots
  const bool masked = M.r_masked[i], replaced = M.r_replaced[i], rnd = M.r_random[i];
  M.labels[i] = masked ? id : M.ignore_index;
  if (replaced) M.ids[i] = M.mask_id;
  else if (rnd) M.ids[i] = M.r_words[i];
}

}  // namespace
}  // namespace lddl

using namespace lddl;

extern "C" int lddl_collate_encode(lddl_ctx* c, void* stream, const uint8_t* d_bytes,
                                   const int64_t* d_a_off, const int64_t* d_b_off,
                                   const int32_t* d_na, const int32_t* d_nb, int32_t batch,
                                   int32_t seq_len, int64_t* d_input_ids, int64_t* d_token_type_ids,
                                   int64_t* d_attention_mask, int64_t* d_special_tokens_mask,
                                   const uint8_t* d_lab_bytes, const int64_t* d_lab_off,
                                   const uint16_t* d_pos, const int64_t* d_pos_off,
                                   int64_t* d_labels, int64_t ignore_index) {
  if (!c) LDDL_FAIL(-1, "null ctx");
  if (batch <= 0 || seq_len <= 0) return 0;
  if (c->tab.special_id[kCls] < 0 || c->tab.special_id[kSep] < 0)
    LDDL_FAIL(-1, "vocab needs [CLS] and [SEP]");
  EncodeArgs E{c->tab, d_bytes, d_a_off, d_b_off, d_na, d_nb, batch, seq_len, d_input_ids,
               d_token_type_ids, d_attention_mask, d_special_tokens_mask, d_lab_bytes, d_lab_off,
               d_pos, d_pos_off, d_labels, ignore_index, 0, {}};
  const size_t lds = sizeof(int32_t) * 2 * (size_t)seq_len * kEncWaves;
  if (lds > 160 * 1024) LDDL_FAIL(-1, "sequence length %d too long for the collate kernel", seq_len);
  hipLaunchKernelGGL(encode_kernel, dim3((unsigned)((batch + kEncWaves - 1) / kEncWaves)),
                     dim3(64 * kEncWaves), lds, as_stream(stream), E);
  LDDL_HIP(hipGetLastError());
  return 0;
}

extern "C" int lddl_mask_dynamic(lddl_ctx* c, void* stream, int64_t* d_input_ids, int64_t* d_labels,
                                 const int64_t* d_special_tokens_mask, const int32_t* d_na,
                                 const int32_t* d_nb, int64_t batch, int64_t seq_len,
                                 float mlm_probability, int64_t ignore_index, int64_t vocab_len,
                                 uint64_t seed, uint64_t counter, const uint8_t* d_r_masked,
                                 const uint8_t* d_r_replaced, const uint8_t* d_r_random,
                                 const int64_t* d_r_words) {
  if (!c) LDDL_FAIL(-1, "null ctx");
  if (!d_special_tokens_mask && (!d_na != !d_nb)) LDDL_FAIL(-1, "need both lengths or neither");
  if (c->tab.special_id[kMask] < 0) LDDL_FAIL(-1, "vocab has no [MASK]");
  const int64_t n = batch * seq_len;
  if (n <= 0) return 0;
  MaskArgs M{d_input_ids, d_labels, d_special_tokens_mask, d_na, d_nb, batch, seq_len,
             mlm_probability, ignore_index, c->tab.special_id[kMask], vocab_len, {}, seed, counter,
             d_r_masked, d_r_replaced, d_r_random, d_r_words};
  for (int k = 0; k < kNumSpecial; ++k) M.special_ids[k] = c->tab.special_id[k];
  hipLaunchKernelGGL(mask_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     as_stream(stream), M);
  LDDL_HIP(hipGetLastError());
  return 0;
}

extern "C" int lddl_collate_encode_masked(lddl_ctx* c, void* stream, const uint8_t* d_bytes,
                                          const int64_t* d_a_off, const int64_t* d_b_off,
                                          const int32_t* d_na, const int32_t* d_nb, int32_t batch,
                                          int32_t seq_len, int64_t* d_input_ids,
                                          int64_t* d_token_type_ids, int64_t* d_attention_mask,
                                          int64_t* d_labels, float mlm_probability,
                                          int64_t ignore_index, int64_t vocab_len, uint64_t seed,
                                          uint64_t counter) {
  if (!c) LDDL_FAIL(-1, "null ctx");
  if (batch <= 0 || seq_len <= 0) return 0;
  if (c->tab.special_id[kCls] < 0 || c->tab.special_id[kSep] < 0 || c->tab.special_id[kMask] < 0)
    LDDL_FAIL(-1, "vocab needs [CLS], [SEP] and [MASK]");
  if (!d_input_ids || !d_token_type_ids || !d_attention_mask || !d_labels)
    LDDL_FAIL(-1, "null output");
  EncodeArgs E{c->tab, d_bytes, d_a_off, d_b_off, d_na, d_nb, batch, seq_len, d_input_ids,
               d_token_type_ids, d_attention_mask, nullptr, nullptr, nullptr, nullptr, nullptr,
               d_labels, ignore_index, 1,
               MaskDraw{mlm_probability, ignore_index, c->tab.special_id[kMask], vocab_len, seed,
                        counter}};
  const size_t lds = sizeof(int32_t) * 2 * (size_t)seq_len * kEncWaves;
  if (lds > 160 * 1024) LDDL_FAIL(-1, "sequence length %d too long for the collate kernel", seq_len);
  hipLaunchKernelGGL(encode_kernel, dim3((unsigned)((batch + kEncWaves - 1) / kEncWaves)),
                     dim3(64 * kEncWaves), lds, as_stream(stream), E);
  LDDL_HIP(hipGetLastError());
  return 0;
}
