// NSP pair construction + static MLM masking on the GPU.
//
// Reference: lddl/dask/bert/pretrain.py
//   _get_documents filtering       89-97   -> compact_* kernels (drop empty sentences / documents)
//   _to_partition_pairs           386-402  -> plan kernel (one wave per partition) + final shuffle
//   create_pairs_from_document    241-365  -> plan_document()
//   _truncate_seq_pair            161-176  -> truncation loop in plan_document()
//   create_masked_lm_predictions  182-238  -> mask decisions in plan_document(), applied by gather
//
// Split into a control plane that touches only integers (sentence lengths, RNG draws) and a data
// plane that moves tokens:
//   plan    one wave per partition. Replay mode reproduces CPython's `random` exactly
//           (random.seed(part_seed[p]) then the reference's draw sequence): the wave executes the
//           sequential algorithm wave-uniformly (every lane computes the same scalars, so control
//           flow never diverges), keeps the MT19937 state in LDS and regenerates it with a
//           64-lane cooperative twist. Output: 32-byte pair descriptors (sentence span + truncation
//           window of A and B) and, with masking, the chosen positions + replacement ids.
//   layout  scans of per-partition pair counts and per-pair token / mask counts (final order =
//           the partition shuffle of pretrain.py:401).
//   gather  one wave per pair: coalesced copy of A and B token spans from the tokenizer output,
//           applying the mask decisions and emitting positions + labels.
#include <vector>

#include "common.h"
#include "ctx.h"
#include "device.h"
#include "lddl_amd.h"
#include "scan.h"

namespace lddl {
namespace {

struct alignas(16) PairDesc {
  int64_t a_ks;     // kept-sentence index where A's chunk starts
  int64_t b_ks;     // kept-sentence index where B's span starts
  int32_t a_front;  // tokens truncated from the front of A's concatenated sentences
  int32_t na;       // tokens kept in A
  int32_t b_front;
  int32_t nb_rn;    // tokens kept in B | is_random_next << 31
};

constexpr int32_t kKeep = -1;  // mask decision "keep the original token" (pretrain.py:215-216)

// ---------------------------------------------------------------------------------------------
// Compaction (pretrain.py:89-97): drop sentences with no pieces, then documents with no sentences
// ---------------------------------------------------------------------------------------------
struct KeepSent {
  const int32_t* len;
  __device__ int64_t operator()(int64_t s) const { return (len[s] & kLenMask) > 0; }
};
struct KeepDoc {
  const int64_t* ks_pos;  // exclusive scan of KeepSent, n_sent+1
  const int64_t* doc_sent_off;
  __device__ int64_t operator()(int64_t d) const {
    return ks_pos[doc_sent_off[d + 1]] > ks_pos[doc_sent_off[d]];
  }
};

__global__ void scatter_sentences_kernel(const int64_t* sent_off, const int32_t* sent_len,
                                         int64_t n_sent, const int64_t* ks_pos, int64_t* ks_start,
                                         int32_t* ks_len) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_sent) return;
  const int32_t l = sent_len[s];
  if ((l & kLenMask) == 0) return;
  const int64_t k = ks_pos[s];
  ks_start[k] = sent_off[s];
  ks_len[k] = l;
}

__global__ void scatter_docs_kernel(const int64_t* doc_sent_off, int64_t n_doc, const int64_t* ks_pos,
                                    const int64_t* kd_pos, int64_t* kd_off) {
  const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (d > n_doc) return;
  if (d == n_doc) { kd_off[kd_pos[n_doc]] = ks_pos[doc_sent_off[n_doc]]; return; }
  if (kd_pos[d + 1] > kd_pos[d]) kd_off[kd_pos[d]] = ks_pos[doc_sent_off[d]];
}

__global__ void part_offsets_kernel(const int64_t* part_doc_off, int64_t n_part, const int64_t* kd_pos,
                                    int64_t* kp_off) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p <= n_part) kp_off[p] = kd_pos[part_doc_off[p]];
}

// ---------------------------------------------------------------------------------------------
// Wave-uniform CPython MT19937 (Modules/_randommodule.c) with the state in LDS.
// ---------------------------------------------------------------------------------------------
constexpr int kN = 624, kM = 397;

struct WaveMT {
  uint32_t* mt;  // LDS [624]
  int mti;

  __device__ void seed_i64(int64_t seed) {  // random.seed(int): init_by_array(abs(seed) limbs)
    if (threadIdx.x == 0) {
      const uint64_t a = seed < 0 ? (uint64_t)(-(seed + 1)) + 1 : (uint64_t)seed;
      const uint32_t key[2] = {(uint32_t)a, (uint32_t)(a >> 32)};
      const int klen = key[1] ? 2 : 1;
      uint32_t prev = 19650218u;
      mt[0] = prev;
      for (int i = 1; i < kN; ++i) {
        prev = 1812433253u * (prev ^ (prev >> 30)) + (uint32_t)i;
        mt[i] = prev;
      }
      int i = 1, j = 0;
      prev = mt[0];
      for (int k = kN; k; --k) {
        const uint32_t v = (mt[i] ^ ((prev ^ (prev >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
        mt[i] = v;
        prev = v;
        ++i;
        ++j;
        if (i >= kN) { mt[0] = mt[kN - 1]; prev = mt[0]; i = 1; }
        if (j >= klen) j = 0;
      }
      for (int k = kN - 1; k; --k) {
        const uint32_t v = (mt[i] ^ ((prev ^ (prev >> 30)) * 1566083941u)) - (uint32_t)i;
        mt[i] = v;
        prev = v;
        ++i;
        if (i >= kN) { mt[0] = mt[kN - 1]; prev = mt[0]; i = 1; }
      }
      mt[0] = 0x80000000u;
    }
    __syncthreads();
    mti = kN;
  }

  __device__ static uint32_t twist1(uint32_t a, uint32_t b, uint32_t c) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
  }

  // all 64 lanes: regenerate the 624-word block in three dependency-free phases
  __device__ void twist() {
    const int l = threadIdx.x;
    for (int i = l; i < kN - kM; i += 64) {  // [0,227): old[i], old[i+1], old[i+397]
      const uint32_t v = twist1(mt[i], mt[i + 1], mt[i + kM]);
      mt[i] = v;
    }
    __syncthreads();
    for (int i = kN - kM + l; i < 2 * (kN - kM); i += 64) {  // [227,454): new[i-227]
      const uint32_t v = twist1(mt[i], mt[i + 1], mt[i - (kN - kM)]);
      mt[i] = v;
    }
    __syncthreads();
    for (int i = 2 * (kN - kM) + l; i < kN - 1; i += 64) {  // [454,623): new[i-227]
      const uint32_t v = twist1(mt[i], mt[i + 1], mt[i - (kN - kM)]);
      mt[i] = v;
    }
    __syncthreads();
    if (l == 0) mt[kN - 1] = twist1(mt[kN - 1], mt[0], mt[kM - 1]);
    __syncthreads();
  }

  __device__ uint32_t u32() {
    if (mti >= kN) {
      twist();
      mti = 0;
    }
    uint32_t y = mt[mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
  __device__ double random() {
    const uint32_t a = u32() >> 5, b = u32() >> 6;
    return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
  }
  __device__ uint32_t randbelow(uint32_t n) {
    const int k = 32 - __clz(n);
    uint32_t r = u32() >> (32 - k);
    while (r >= n) r = u32() >> (32 - k);
    return r;
  }
  __device__ int64_t randint(int64_t a, int64_t b) { return a + randbelow((uint32_t)(b - a + 1)); }
};

struct PlanArgs {
  // kept corpus
  const int64_t* ks_start;
  const int32_t* ks_len;
  const int64_t* kd_off;
  const int64_t* kp_off;
  const int32_t* ids;
  const int64_t* part_seed;
  // params
  int32_t seq, dup, masking, vocab_size, cls_id, sep_id, mask_id, max_pred;
  double short_seq_prob, ratio;
  // outputs, slot base of partition p = dup * kd_off[kp_off[p]]
  PairDesc* desc;
  int32_t* order;      // per slot: creation index at final position
  int32_t* nmask;      // per slot
  uint16_t* mpos;      // per slot * max_pred
  int32_t* mtok;       // per slot * max_pred
  int64_t* part_npairs;
};

__device__ inline int32_t slen(const PlanArgs& A, int64_t k) { return A.ks_len[k] & kLenMask; }

// token j (0-based) of the span that starts at kept sentence k0 (sequential walk; slow path only)
__device__ int32_t span_token(const PlanArgs& A, int64_t k0, int64_t j) {
  for (int64_t k = k0;; ++k) {
    const int32_t l = slen(A, k);
    if (j < l) return A.ids[A.ks_start[k] + j];
    j -= l;
  }
}

__global__ void __launch_bounds__(64) plan_replay_kernel(PlanArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  WaveMT rng{reinterpret_cast<uint32_t*>(smem), kN};
  uint16_t* cand = reinterpret_cast<uint16_t*>(smem + 4 * kN);              // [seq]
  uint16_t* tpos = cand + ((A.seq + 7) & ~7);                                // [max_pred]
  int32_t* ttok = reinterpret_cast<int32_t*>(tpos + ((A.max_pred + 7) & ~7));  // [max_pred]
  const int p = blockIdx.x;
  const int lane = threadIdx.x;
  const bool leader = lane == 0;
  rng.seed_i64(A.part_seed[p]);
  const int64_t d0 = A.kp_off[p], nd = A.kp_off[p + 1] - d0;
  const int64_t base = (int64_t)A.dup * A.kd_off[d0];
  const int32_t max_num = A.seq - 3;
  int64_t np = 0;
  for (int dp = 0; dp < A.dup; ++dp) {
    for (int64_t di = 0; di < nd; ++di) {
      const int64_t s0 = A.kd_off[d0 + di], ns = A.kd_off[d0 + di + 1] - s0;
      int32_t target = max_num;
      if (rng.random() < A.short_seq_prob) target = (int32_t)rng.randint(2, max_num);
      int64_t chunk0 = 0, chunk_n = 0, cur_len = 0;
      for (int64_t i = 0; i < ns; ++i) {
        if (chunk_n == 0) chunk0 = i;
        ++chunk_n;
        cur_len += slen(A, s0 + i);
        if (!(i == ns - 1 || cur_len >= target)) continue;
        const int64_t a_end = chunk_n >= 2 ? rng.randint(1, chunk_n - 1) : 1;
        int64_t la = 0;
        int32_t flags = 0;
        for (int64_t j = chunk0; j < chunk0 + a_end; ++j) {
          la += slen(A, s0 + j);
          flags |= A.ks_len[s0 + j];
        }
        int64_t lb = 0, b_ks;
        int32_t rn = 0;
        if (chunk_n == 1 || rng.random() < 0.5) {
          rn = 1;
          const int64_t target_b = target - la;
          int64_t rd = 0;
          for (int t = 0; t < 10; ++t) {
            rd = rng.randint(0, nd - 1);
            if (rd != di) break;
          }
          if (rd == di) rn = 0;
          const int64_t r0 = A.kd_off[d0 + rd], rns = A.kd_off[d0 + rd + 1] - r0;
          const int64_t rstart = rng.randint(0, rns - 1);
          b_ks = r0 + rstart;
          for (int64_t j = rstart; j < rns; ++j) {
            lb += slen(A, r0 + j);
            flags |= A.ks_len[r0 + j];
            if (lb >= target_b) break;
          }
          i -= chunk_n - a_end;
        } else {
          b_ks = s0 + chunk0 + a_end;
          for (int64_t j = chunk0 + a_end; j < chunk0 + chunk_n; ++j) {
            lb += slen(A, s0 + j);
            flags |= A.ks_len[s0 + j];
          }
        }
        // _truncate_seq_pair
        int32_t a_front = 0, b_front = 0, na = (int32_t)la, nb = (int32_t)lb;
        while (na + nb > max_num) {
          const bool front = rng.random() < 0.5;
          if (na > nb) { a_front += front; --na; }
          else { b_front += front; --nb; }
        }
        const int64_t slot = base + np;
        if (leader) A.desc[slot] = PairDesc{s0 + chunk0, b_ks, a_front, na, b_front,
                                            nb | (int32_t)((uint32_t)rn << 31)};
        if (A.masking) {
          // candidates: every position of [CLS] A [SEP] B [SEP] whose token is not [CLS]/[SEP]
          int32_t nc = na + nb;
          if (flags & kLenHasClsSep) {  // literal [CLS]/[SEP] inside A or B: inspect tokens
            int32_t c = 0;
            for (int32_t t = 0; t < na + nb; ++t) {
              const int32_t tok = t < na ? span_token(A, s0 + chunk0, a_front + t)
                                         : span_token(A, b_ks, b_front + (t - na));
              if (tok != A.cls_id && tok != A.sep_id) {
                if (leader) cand[c] = (uint16_t)(t < na ? t + 1 : t + 2);
                ++c;
              }
            }
            nc = c;
          } else {
            for (int32_t k = lane; k < nc; k += 64) cand[k] = (uint16_t)(k < na ? k + 1 : k + 2);
          }
          __syncthreads();
          for (int32_t k = nc - 1; k > 0; --k) {  // random.shuffle(cand_indexes)
            const uint32_t j = rng.randbelow((uint32_t)k + 1);
            if (leader) {
              const uint16_t t = cand[k];
              cand[k] = cand[j];
              cand[j] = t;
            }
          }
          const double prod = (double)(na + nb + 3) * A.ratio;
          int32_t num = (int32_t)rint(prod);  // Python round(): half to even
          if (num < 1) num = 1;
          if (num > nc) num = nc;
          for (int32_t c = 0; c < num; ++c) {
            int32_t tok;
            if (rng.random() < 0.8) tok = A.mask_id;
            else if (rng.random() < 0.5) tok = kKeep;
            else tok = (int32_t)rng.randint(0, A.vocab_size - 1);
            if (leader) {
              tpos[c] = cand[c];
              ttok[c] = tok;
            }
          }
          __syncthreads();
          // sorted(masked_lms, key=index): rank sort (positions are distinct)
          for (int32_t c = lane; c < num; c += 64) {
            const uint16_t v = tpos[c];
            int32_t r = 0;
            for (int32_t o = 0; o < num; ++o) r += tpos[o] < v;
            A.mpos[slot * A.max_pred + r] = v;
            A.mtok[slot * A.max_pred + r] = ttok[c];
          }
          if (leader) A.nmask[slot] = num;
          __syncthreads();
        }
        ++np;
        chunk_n = 0;
        cur_len = 0;
      }
    }
  }
  // random.shuffle(partition_pairs): order[base + k] = creation index of the pair at position k
  if (leader) {
    int32_t* ord = A.order + base;
    for (int64_t k = 0; k < np; ++k) ord[k] = (int32_t)k;
  }
  for (int64_t k = np - 1; k > 0; --k) {
    const uint32_t j = rng.randbelow((uint32_t)k + 1);
    if (leader) {
      int32_t* ord = A.order + base;
      const int32_t t = ord[k];
      ord[k] = ord[j];
      ord[j] = t;
    }
  }
  if (leader) A.part_npairs[p] = np;
}

// ---------------------------------------------------------------------------------------------
// layout + gather
// ---------------------------------------------------------------------------------------------
__global__ void map_pairs_kernel(const int64_t* kd_off, const int64_t* kp_off, int32_t dup,
                                 const int64_t* part_pair_base, const int32_t* order, int64_t* src) {
  const int p = blockIdx.x;
  const int64_t base = (int64_t)dup * kd_off[kp_off[p]];
  const int64_t q0 = part_pair_base[p], n = part_pair_base[p + 1] - q0;
  for (int64_t k = threadIdx.x; k < n; k += blockDim.x) src[q0 + k] = base + order[base + k];
}

struct PairTokens {
  const int64_t* src;
  const PairDesc* desc;
  __device__ int64_t operator()(int64_t q) const {
    const PairDesc d = desc[src[q]];
    return (int64_t)d.na + (d.nb_rn & 0x7FFFFFFF);
  }
};
struct Identity {
  const int64_t* v;
  __device__ int64_t operator()(int64_t i) const { return v[i]; }
};
struct PairMasks {
  const int64_t* src;
  const int32_t* nmask;
  __device__ int64_t operator()(int64_t q) const { return nmask[src[q]]; }
};

struct GatherArgs {
  const int64_t* ks_start;
  const int32_t* ks_len;
  const int32_t* ids;
  const int64_t* src;
  const PairDesc* desc;
  const int32_t* nmask;
  const uint16_t* mpos;
  const int32_t* mtok;
  int32_t max_pred, masking;
  int64_t n_pairs;
  const int64_t* tok_off;
  const int64_t* pos_off;
  int32_t* out_tok;
  int32_t* len_a;
  uint8_t* is_rn;
  uint16_t* out_pos;
  int32_t* out_lab;
};

constexpr int kGatherWaves = 4;
constexpr int kMaxPredLds = 1024;

// Copy `count` tokens of the span starting at kept sentence k0 after skipping `front` tokens to
// out[0..count); output index t has sequence position pos0 + t.
__device__ void copy_span(const GatherArgs& G, int64_t k0, int32_t front, int32_t count, int32_t* out,
                          int32_t pos0, const uint16_t* mp, const int32_t* mt, int32_t nm,
                          int32_t* lab) {
  int32_t t = 0;
  const int lane = lane_id();
  for (int64_t k = k0; t < count; ++k) {
    const int32_t l = G.ks_len[k] & kLenMask;
    if (front >= l) { front -= l; continue; }
    const int32_t take = min(l - front, count - t);
    const int32_t* srcp = G.ids + G.ks_start[k] + front;
    for (int32_t x = lane; x < take; x += 64) {
      int32_t tok = srcp[x];
      if (nm) {
        const int32_t pos = pos0 + t + x;
        int lo = 0, hi = nm;  // binary search in the sorted masked positions
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (mp[mid] < pos) lo = mid + 1; else hi = mid;
        }
        if (lo < nm && mp[lo] == pos) {
          lab[lo] = tok;
          if (mt[lo] != kKeep) tok = mt[lo];
        }
      }
      out[t + x] = tok;
    }
    t += take;
    front = 0;
  }
}

__global__ void __launch_bounds__(64 * kGatherWaves) gather_kernel(GatherArgs G) {
  __shared__ uint16_t s_pos[kGatherWaves][kMaxPredLds];
  __shared__ int32_t s_tok[kGatherWaves][kMaxPredLds];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * kGatherWaves + w;
  const bool active = q < G.n_pairs;
  const int64_t slot = active ? G.src[q] : 0;
  int32_t nm = 0;
  int32_t* lab = nullptr;
  if (G.masking && active) {
    nm = G.nmask[slot];
    for (int j = lane; j < nm; j += 64) {
      const uint16_t pv = G.mpos[slot * G.max_pred + j];
      s_pos[w][j] = pv;
      s_tok[w][j] = G.mtok[slot * G.max_pred + j];
      G.out_pos[G.pos_off[q] + j] = pv;
    }
    lab = G.out_lab + G.pos_off[q];
  }
  __syncthreads();  // masked positions visible to every lane of the wave
  if (!active) return;
  const PairDesc d = G.desc[slot];
  const int32_t nb = d.nb_rn & 0x7FFFFFFF;
  int32_t* out = G.out_tok + G.tok_off[q];
  copy_span(G, d.a_ks, d.a_front, d.na, out, 1, s_pos[w], s_tok[w], nm, lab);
  copy_span(G, d.b_ks, d.b_front, nb, out + d.na, d.na + 2, s_pos[w], s_tok[w], nm, lab);
  if (lane == 0) {
    G.len_a[q] = d.na;
    G.is_rn[q] = (uint8_t)((uint32_t)d.nb_rn >> 31);
  }
}

}  // namespace
}  // namespace lddl

using namespace lddl;

// Device-resident plan of one batch of partitions (library-owned temporaries).
struct lddl_pairs {
  int device = 0;
  int32_t masking = 0, max_pred = 0;
  int64_t n_part = 0, n_pairs = 0, n_tokens = 0, n_masked = 0, n_kept_sent = 0, n_kept_doc = 0;
  std::vector<void*> allocs;
  // views
  int64_t *ks_start = nullptr, *kd_off = nullptr, *kp_off = nullptr;
  int32_t* ks_len = nullptr;
  const int32_t* ids = nullptr;
  PairDesc* desc = nullptr;
  int32_t *order = nullptr, *nmask = nullptr, *mtok = nullptr;
  uint16_t* mpos = nullptr;
  int64_t *src = nullptr, *tok_off = nullptr, *pos_off = nullptr;

  template <typename T>
  int alloc(T** p, int64_t n, hipStream_t st) {
    LDDL_HIP(hipMallocAsync((void**)p, sizeof(T) * (size_t)(n > 0 ? n : 1), st));
    allocs.push_back(*p);
    return 0;
  }
  void release(hipStream_t st) {
    for (void* p : allocs) (void)hipFreeAsync(p, st);
    allocs.clear();
  }
};

#define TRY(x)                     \
  do {                             \
    int rc_ = (x);                 \
    if (rc_) {                     \
      P->release(st);              \
      delete P;                    \
      return rc_;                  \
    }                              \
  } while (0)

extern "C" int lddl_pairs_plan(lddl_ctx* c, void* stream, const lddl_pair_params* prm,
                               const int64_t* d_sent_off, const int32_t* d_ids,
                               const int32_t* d_sent_len, int64_t n_sent,
                               const int64_t* d_doc_sent_off, int64_t n_doc,
                               const int64_t* d_part_doc_off, const int64_t* d_part_seed,
                               int64_t n_part, lddl_pairs** out, int64_t* counts) {
  *out = nullptr;
  if (!c || !prm) LDDL_FAIL(-1, "null argument");
  if (prm->seq < 5 || prm->seq > 65535) LDDL_FAIL(-1, "target_seq_length %d out of range", prm->seq);
  if (prm->dup < 1) LDDL_FAIL(-1, "duplicate_factor must be >= 1");
  if (prm->rng != LDDL_RNG_REPLAY) LDDL_FAIL(-1, "rng mode %d not available", prm->rng);
  const int32_t cls = c->tab.special_id[kCls], sep = c->tab.special_id[kSep],
                msk = c->tab.special_id[kMask];
  if (prm->masking && (cls < 0 || sep < 0 || msk < 0))
    LDDL_FAIL(-1, "static masking needs [CLS] [SEP] [MASK] in the vocab");
  hipStream_t st = as_stream(stream);
  auto* P = new lddl_pairs();
  P->device = c->device;
  P->n_part = n_part;
  P->masking = prm->masking;
  P->ids = d_ids;
  int64_t *ks_pos, *kd_pos, *scratch, *part_npairs, *part_base;
  const int64_t nscr = scan_scratch_elems(std::max(n_sent, n_doc) + n_part + 1);
  TRY(P->alloc(&scratch, nscr, st));
  // compaction
  TRY(P->alloc(&ks_pos, n_sent + 1, st));
  if (scan_exclusive(KeepSent{d_sent_len}, n_sent, ks_pos, scratch, st) != hipSuccess)
    TRY(-100);
  TRY(P->alloc(&kd_pos, n_doc + 1, st));
  if (scan_exclusive(KeepDoc{ks_pos, d_doc_sent_off}, n_doc, kd_pos, scratch, st) != hipSuccess)
    TRY(-100);
  int64_t h_counts[2];
  LDDL_HIP(hipMemcpyAsync(&h_counts[0], ks_pos + n_sent, 8, hipMemcpyDeviceToHost, st));
  LDDL_HIP(hipMemcpyAsync(&h_counts[1], kd_pos + n_doc, 8, hipMemcpyDeviceToHost, st));
  LDDL_HIP(hipStreamSynchronize(st));
  P->n_kept_sent = h_counts[0];
  P->n_kept_doc = h_counts[1];
  TRY(P->alloc(&P->ks_start, P->n_kept_sent, st));
  TRY(P->alloc(&P->ks_len, P->n_kept_sent, st));
  TRY(P->alloc(&P->kd_off, P->n_kept_doc + 1, st));
  TRY(P->alloc(&P->kp_off, n_part + 1, st));
  if (n_sent)
    hipLaunchKernelGGL(scatter_sentences_kernel, dim3((unsigned)((n_sent + 255) / 256)), dim3(256), 0,
                       st, d_sent_off, d_sent_len, n_sent, ks_pos, P->ks_start, P->ks_len);
  hipLaunchKernelGGL(scatter_docs_kernel, dim3((unsigned)((n_doc + 256) / 256)), dim3(256), 0, st,
                     d_doc_sent_off, n_doc, ks_pos, kd_pos, P->kd_off);
  hipLaunchKernelGGL(part_offsets_kernel, dim3((unsigned)((n_part + 256) / 256)), dim3(256), 0, st,
                     d_part_doc_off, n_part, kd_pos, P->kp_off);
  LDDL_HIP(hipGetLastError());
  // plan
  const int64_t slots = (int64_t)prm->dup * P->n_kept_sent;
  int32_t max_pred = 0;
  if (prm->masking) {
    max_pred = (int32_t)rint((double)prm->seq * prm->masked_lm_ratio);
    if (max_pred < 1) max_pred = 1;
    if (max_pred > prm->seq) max_pred = prm->seq;
    if (max_pred > kMaxPredLds) TRY((set_error("masked_lm_ratio * seq too large"), -1));
  }
  P->max_pred = max_pred;
  TRY(P->alloc(&P->desc, slots, st));
  TRY(P->alloc(&P->order, slots, st));
  TRY(P->alloc(&part_npairs, n_part + 1, st));
  if (prm->masking) {
    TRY(P->alloc(&P->nmask, slots, st));
    TRY(P->alloc(&P->mpos, slots * max_pred, st));
    TRY(P->alloc(&P->mtok, slots * max_pred, st));
  }
  PlanArgs A{P->ks_start, P->ks_len, P->kd_off, P->kp_off, d_ids, d_part_seed,
             prm->seq, prm->dup, prm->masking, c->vocab_size, cls, sep, msk, max_pred,
             prm->short_seq_prob, prm->masked_lm_ratio,
             P->desc, P->order, P->nmask, P->mpos, P->mtok, part_npairs};
  const size_t lds = 4 * kN + 2 * ((prm->seq + 7) & ~7) + 2 * ((max_pred + 7) & ~7) + 4 * max_pred + 16;
  if (n_part)
    hipLaunchKernelGGL(plan_replay_kernel, dim3((unsigned)n_part), dim3(64), lds, st, A);
  LDDL_HIP(hipGetLastError());
  // layout
  TRY(P->alloc(&part_base, n_part + 1, st));
  if (scan_exclusive(Identity{part_npairs}, n_part, part_base, scratch, st) != hipSuccess) TRY(-100);
  LDDL_HIP(hipMemcpyAsync(&P->n_pairs, part_base + n_part, 8, hipMemcpyDeviceToHost, st));
  LDDL_HIP(hipStreamSynchronize(st));
  const int64_t npairs = P->n_pairs;
  TRY(P->alloc(&P->src, npairs, st));
  TRY(P->alloc(&P->tok_off, npairs + 1, st));
  if (n_part)
    hipLaunchKernelGGL(map_pairs_kernel, dim3((unsigned)n_part), dim3(256), 0, st, P->kd_off,
                       P->kp_off, prm->dup, part_base, P->order, P->src);
  int64_t* scr2;
  TRY(P->alloc(&scr2, scan_scratch_elems(npairs), st));
  if (scan_exclusive(PairTokens{P->src, P->desc}, npairs, P->tok_off, scr2, st) != hipSuccess)
    TRY(-100);
  LDDL_HIP(hipMemcpyAsync(&P->n_tokens, P->tok_off + npairs, 8, hipMemcpyDeviceToHost, st));
  if (prm->masking) {
    TRY(P->alloc(&P->pos_off, npairs + 1, st));
    if (scan_exclusive(PairMasks{P->src, P->nmask}, npairs, P->pos_off, scr2, st) != hipSuccess)
      TRY(-100);
    LDDL_HIP(hipMemcpyAsync(&P->n_masked, P->pos_off + npairs, 8, hipMemcpyDeviceToHost, st));
  }
  LDDL_HIP(hipStreamSynchronize(st));
  if (counts) {
    counts[0] = P->n_pairs;
    counts[1] = P->n_tokens;
    counts[2] = P->n_masked;
    counts[3] = P->n_kept_sent;
    counts[4] = P->n_kept_doc;
  }
  *out = P;
  return 0;
}

extern "C" int lddl_pairs_emit(lddl_pairs* P, void* stream, int32_t* d_tokens, int64_t* d_tok_off,
                               int32_t* d_len_a, uint8_t* d_is_rn, uint16_t* d_pos, int32_t* d_lab,
                               int64_t* d_pos_off) {
  if (!P) LDDL_FAIL(-1, "null plan");
  hipStream_t st = as_stream(stream);
  if (P->n_pairs == 0) return 0;
  GatherArgs G{P->ks_start, P->ks_len, P->ids, P->src, P->desc, P->nmask, P->mpos, P->mtok,
               P->max_pred, P->masking, P->n_pairs, P->tok_off, P->pos_off, d_tokens, d_len_a,
               d_is_rn, d_pos, d_lab};
  const int64_t grid = (P->n_pairs + kGatherWaves - 1) / kGatherWaves;
  hipLaunchKernelGGL(gather_kernel, dim3((unsigned)grid), dim3(64 * kGatherWaves), 0, st, G);
  LDDL_HIP(hipGetLastError());
  if (d_tok_off)
    LDDL_HIP(hipMemcpyAsync(d_tok_off, P->tok_off, 8 * (P->n_pairs + 1), hipMemcpyDeviceToDevice, st));
  if (d_pos_off && P->masking)
    LDDL_HIP(hipMemcpyAsync(d_pos_off, P->pos_off, 8 * (P->n_pairs + 1), hipMemcpyDeviceToDevice, st));
  return 0;
}

extern "C" int lddl_pairs_destroy(lddl_pairs* P, void* stream) {
  if (!P) return 0;
  P->release(as_stream(stream));
  delete P;
  return 0;
}
