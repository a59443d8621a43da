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
#include <algorithm>
#include <cstdio>
#include <vector>

#include <cstdlib>
#include <cstring>

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

// Replay masking, per planner slot: where the pair's decisions (mask pool, entries moff8 * 8 ..)
// and shuffle draws (draw pool, joff16 * 16 ..) are, and how many. One 16-byte record, one store.
struct alignas(16) SlotPool {
  uint32_t moff8;   // mask-pool offset / 8 (regions are 8-entry aligned)
  uint32_t joff16;  // draw-pool offset / 16 (regions are 16-entry aligned)
  int32_t nmask;    // num_to_predict
  int32_t ncand;    // candidates (len(A) + len(B) minus literal [CLS]/[SEP])
};

constexpr int32_t kKeep = -1;  // mask decision "keep the original token" (pretrain.py:215-216)

// Diagnostic build only (-DLDDL_STAMPS): per-region s_memtime sums of the planner.
#ifdef LDDL_STAMPS
constexpr int kStampRegions = 8;
#define STAMP_T() __builtin_amdgcn_s_memtime()
#define STAMP_ADD(r, t0)                   \
  do {                                     \
    const uint64_t t1_ = STAMP_T();        \
    st_acc[r] += t1_ - (t0);               \
    t0 = t1_;                              \
  } while (0)
#else
#define STAMP_T() 0ull
#define STAMP_ADD(r, t0) ((void)0)
#endif

// ---------------------------------------------------------------------------------------------
// Compaction (pretrain.py:89-97): drop sentences with no pieces, then documents with no sentences
// ---------------------------------------------------------------------------------------------
struct KeepSent {
  const int32_t* len;
  __device__ int64_t operator()(int64_t s) const { return (len[s] & kLenMask) > 0; }
};
// both sentence scans in one pass: kept-sentence index and token offset. A dropped sentence has
// no tokens, so the token scan over all sentences, read at the kept ones, is the kept-token scan.
struct SentCounts {
  const int32_t* len;
  __device__ Sum2 operator()(int64_t s) const {
    const int32_t l = len[s] & kLenMask;
    return Sum2{l > 0 ? 1 : 0, l};
  }
};
struct KeepDoc {
  const int64_t* ks_pos;  // exclusive scan of KeepSent, n_sent+1
  const int64_t* doc_sent_off;
  __device__ int64_t operator()(int64_t d) const {
    return ks_pos[doc_sent_off[d + 1]] > ks_pos[doc_sent_off[d]];
  }
};

// kept sentence k = ks_pos[s]: its text start, length and token offset kscan[k] = tok_pos[s]
// (kscan[n_kept] = the total, from thread n_sent)
__global__ void scatter_sentences_kernel(const int64_t* sent_off, const int32_t* sent_len,
                                         int64_t n_sent, const int64_t* ks_pos, const int64_t* tok_pos,
                                         int64_t* ks_start, int32_t* ks_len, int64_t* kscan) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s > n_sent) return;
  if (s == n_sent) {
    kscan[ks_pos[n_sent]] = tok_pos[n_sent];
    return;
  }
  const int32_t l = sent_len[s];
  if ((l & kLenMask) == 0) return;
  const int64_t k = ks_pos[s];
  ks_start[k] = sent_off[s];
  ks_len[k] = l;
  kscan[k] = tok_pos[s];
}

__global__ void scatter_docs_kernel(const int64_t* doc_sent_off, int64_t n_doc, const int64_t* ks_pos,
                                    const int64_t* kd_pos, int64_t* kd_off) {
  const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (d > n_doc) return;
  if (d == n_doc) { kd_off[kd_pos[n_doc]] = ks_pos[doc_sent_off[n_doc]]; return; }
  if (kd_pos[d + 1] > kd_pos[d]) kd_off[kd_pos[d]] = ks_pos[doc_sent_off[d]];
}

__global__ void part_offsets_kernel(const int64_t* part_doc_off, int64_t n_part, const int64_t* kd_pos,
                                    int64_t* kp_off, unsigned long long* max_docs) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p <= n_part) kp_off[p] = kd_pos[part_doc_off[p]];
  if (p < n_part)  // kept documents of the largest partition (the planner's LDS table choice)
    atomicMax(max_docs, (unsigned long long)(kd_pos[part_doc_off[p + 1]] - kd_pos[part_doc_off[p]]));
}

// ---------------------------------------------------------------------------------------------
// Wave-uniform CPython MT19937 (Modules/_randommodule.c).
// Raw state and the tempered 624-word block live in LDS; draws are served from a register
// window (lane l holds word wbase+l) through readlane, so a draw costs a few instructions.
// Every lane executes the same sequential algorithm with identical scalars (uniform control
// flow); only parallel phases (twist, temper, speculative shuffle draws) use the lanes.
// ---------------------------------------------------------------------------------------------
constexpr int kN = 624, kM = 397;
constexpr int kLook = 64;  // MT words of look-ahead past the block (WaveRng)
constexpr int64_t kPoolChunk = 4096;  // mask pool entries reserved per atomic

__device__ inline int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ inline uint32_t rdlane(uint32_t v, int idx) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, uni(idx));
}
__device__ inline uint32_t temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

struct WaveRng {
  // LDS: the raw 624-word block followed by kLook words of look-ahead, the next block's first
  // words (next[i] = twist1(cur[i], cur[i+1], cur[i+397]) for i < 227 depends on the current
  // block alone). mti indexes that extended stream: a window starting at mti < 624 may read up to
  // kLook words past it without a block check, and the twist runs when a window or a register
  // refill starts at mti >= 624 (mti -= 624 afterwards).
  uint32_t* mt;
  int mti;       // next word (uniform), < kN + kLook
  int wbase;     // register window base (uniform)
  int wend;      // wbase + 64 while the register window is valid, 0 when stale (uniform)
  uint32_t win;  // this lane's tempered word temper(mt[wbase + lane])
#ifdef LDDL_STAMPS
  uint64_t n_pass = 0, n_win = 0;  // diagnostics: Jacobi passes / Fisher-Yates windows
#endif

  __device__ static uint32_t twist1(uint32_t a, uint32_t b, uint32_t c) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
  }

  // Regenerate the block in place with all 64 lanes: ten straight-line rounds of 64 consecutive
  // words (no exec-mask loops), then the look-ahead. Word i reads old[i], old[i+1] and old[i+397]
  // (i < 227) or new[i-227], written three rounds earlier; a round reads before it writes, and
  // one wave's LDS operations complete in order, so the rounds need only a compiler fence. Word
  // 623 reads "old[624]" = the look-ahead word 0 = new[0] (seed_i64 sets it for the first block);
  // round 9's lanes past 623 write scratch into the look-ahead, which the last round overwrites.
  __device__ void twist() {
    const int l = threadIdx.x;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      const int i = 64 * r + l;
      const int ci = r < 3 ? i + kM : r > 3 ? i - (kN - kM) : (l < kN - kM - 192 ? i + kM : i - (kN - kM));
      const uint32_t v = twist1(mt[i], mt[i + 1], mt[ci]);
      mt[i] = v;
      __asm__ volatile("" ::: "memory");
    }
    mt[kN + l] = twist1(mt[l], mt[l + 1], mt[l + kM]);  // look-ahead: next block's words 0..63
    __asm__ volatile("" ::: "memory");
    mti -= kN;
    wbase = -1024;
    wend = 0;
  }
  __device__ void ensure() {
    if (mti >= kN) twist();
  }

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
      mt[kN] = twist1(mt[0], mt[1], mt[kM]);  // look-ahead word 0 (= the first twist's new[0])
    }
    __syncthreads();
    mti = kN;  // CPython leaves index = N after seeding: the first draw twists
    wbase = -1024;
    wend = 0;
  }

  // out of line: runs once per 64 draws (window load) or per 624 draws (twist)
  __device__ void refill() {
    ensure();
    wbase = mti;
    wend = mti + 64;
    win = temper(mt[mti + (int)threadIdx.x]);
  }
  __device__ uint32_t u32() {
    if (mti >= wend) refill();  // one scalar compare per draw
    const uint32_t v = rdlane(win, mti - wbase);
    mti = uni(mti + 1);
    return v;
  }
  // Fisher-Yates draws of random.shuffle over n items: j_i = _randbelow(i+1), i = n-1 .. 1,
  // delivered as sink(off, j) by every lane of every window: off = i for the lane whose word
  // is drawn for step i and accepted, 0 for every other lane (rejected words, words past the
  // end; index 0 of a draw array is never read, so the sink stores unconditionally - no
  // exec-mask branch per window). Wave-parallel over a window of 64 words (lane t holds word t).
  // Word t of the window is drawn for step i_t = s0 - t + R_t (R_t = rejections before t) and
  // rejected iff (w_t >> (32 - bit_length(i_t + 1))) > i_t, i.e. with u = i + 1 (the draw's
  // bound) iff (w_t >> clz(u)) >= u. R is the fixed point of R_t = #{v < t : rejected under
  // R_v}, found by Jacobi iteration on ballots: the recurrence is causal, so every pass fixes at
  // least the first wrong word. Words past the last step (u <= 1) come after every valid word
  // and do not affect their R; they are held "accepted" (a verdict that followed their R would
  // keep changing and cost passes: 11.7 instead of ~5 per window), and the first of them ends
  // the shuffle. The window's bookkeeping is branch-free scalar work (s_ff1 / s_bcnt1).
  template <typename Sink>
  __device__ void fy_draws(int32_t n, Sink sink) {
    const int lane = threadIdx.x;
    int32_t s0 = n - 1;  // next step (uniform); n < 2^30 (host-checked)
    while (s0 >= 1) {
      ensure();
      const uint32_t w = temper(mt[mti + lane]);
      const int32_t u1 = s0 + 1 - lane;
      // Jacobi start: ~0.3 rejections per word (any start converges to the same fixed point,
      // the left-most wrong word being fixed by every pass; simulated: 5.3 -> 4.8 passes per
      // window at target_seq_length 128)
      int32_t R = (lane * 77) >> 8;
      uint32_t x;
      uint64_t rej;
      // Convergence is tested on the rejection masks (one scalar 64-bit compare): from the second
      // pass on, R = popc_below(previous mask), so equal masks give equal R in every lane (bit 63
      // moves no R: at most one extra pass). The loop carries no vector compare and no R copy.
      if (s0 >= 64) {  // every word of the window has a step (u >= 2)
        auto pass = [&]() {
          const int32_t u = u1 + R;
          x = w >> __clz((uint32_t)u);
#ifdef LDDL_STAMPS
          ++n_pass;
#endif
          return ballot(x >= (uint32_t)u);
        };
        uint64_t prev = pass();
        R = (int32_t)popc_below(prev);
        rej = pass();
        while (rej != prev) {
          prev = rej;
          R = (int32_t)popc_below(rej);
          rej = pass();
        }
      } else {  // words past the last step (u <= 1) are held "accepted", so they settle at once
        auto pass = [&]() {
          const int32_t u = u1 + R;
          x = w >> (__clz((uint32_t)u) & 31);
#ifdef LDDL_STAMPS
          ++n_pass;
#endif
          return ballot(x >= (uint32_t)u) & ballot(u > 1);
        };
        uint64_t prev = pass();
        R = (int32_t)popc_below(prev);
        rej = pass();
        while (rej != prev) {
          prev = rej;
          R = (int32_t)popc_below(rej);
          rej = pass();
        }
      }
#ifdef LDDL_STAMPS
      ++n_win;
#endif
      const int32_t i = u1 + R - 1;  // the lane's step (<= 0 past the end)
      // (the verdict is recomputed here rather than carried out of the loop as a lane mask)
      sink(x > (uint32_t)i ? 0 : max(i, 0), x);
      // the shuffle ends at the first word past the last step (E); words < E are consumed. After
      // such a window s0 - (64 - popc(rej)) <= 0, since the held words count as accepted.
      const uint64_t fin = ballot(i < 1);
      mti = uni(mti + (fin ? (int)__ffsll((unsigned long long)fin) - 1 : 64));
      s0 -= 64 - (int32_t)__popcll(rej);
    }
    wbase = -1024;
    wend = 0;  // the register window is stale
  }
  // _truncate_seq_pair draws (pretrain.py:161-176). T = na + nb - max_num trims; trim t hits A
  // iff A is the longer side at that point, which has a closed form: with d = na - nb the first
  // |d| trims hit the longer side, then B and A alternate starting with B (ties trim B). Each
  // trim is from the front iff random() < 0.5, i.e. iff the first of its two words is < 2^31, so
  // 32 trims (64 words, the look-ahead) resolve per wave pass with two ballots.
  __device__ void trunc_draws(int32_t& na, int32_t& nb, int32_t max_num, int32_t& a_front,
                              int32_t& b_front) {
    const int32_t T = na + nb - max_num;
    if (T <= 0) return;
    const int32_t d = na - nb, ad = d < 0 ? -d : d;
    const int lane = threadIdx.x;
    for (int32_t done = 0; done < T;) {
      ensure();
      const int32_t cnt = min(T - done, 32);
      const int32_t t = done + lane;
      // random() < 0.5 <=> the tempered first word's top bit is clear; tempering is linear over
      // GF(2) and that bit is the parity of raw bits 31, 27, 24 and 16
      // (every lane reads: mti + 126 stays inside the LDS block; lanes >= cnt are masked off
      // by the scalar lane mask, not by an exec-mask branch)
      const uint32_t par = __popc(mt[mti + 2 * lane] & 0x89010000u) & 1u;
      const uint64_t F = ballot(par == 0) & ((1ull << cnt) - 1);  // cnt <= 32
      const int32_t x = t - ad;
      const uint64_t S = ballot(t < d) | (ballot(x >= 0) & ballot((x & 1) != 0));
      a_front += __popcll(F & S);
      b_front += __popcll(F & ~S);
      mti = uni(mti + 2 * cnt);
      done += cnt;
    }
    wbase = -1024;
    wend = 0;
    const int32_t nA = (d > 0 ? min(d, T) : 0) + (T > ad ? (T - ad) / 2 : 0);
    na -= nA;
    nb -= T - nA;
  }

  // Decisions of create_masked_lm_predictions (pretrain.py:208-221) for cnt masked tokens:
  // random() < 0.8 -> [MASK]; else random() < 0.5 -> keep; else vocab_words[randint(0, V-1)].
  // Lane t tabulates the decision and word count of a token whose first word is mti + t (only
  // decisions whose words lie in the 64-word look-ahead); the chain of decision starts p_0 = 0,
  // p_{k+1} = p_k + len[p_k] is then resolved for every k at once by pointer doubling
  // (ds_bpermute), so lane k learns where decision k starts (a window holds <= 32 decisions).
  // cnt <= 64; returns decision `lane` in each lane < cnt.
  __device__ int32_t mask_decisions(int cnt, uint64_t lt08, int32_t V, int32_t mask_id) {
    const int lane = threadIdx.x;
    const int kV = 32 - __clz((uint32_t)V);
    int32_t res = 0;
    int c = 0;
    while (c < cnt) {
      ensure();
      // word t + j of the window reaches lane t by j whole-wave DPP shifts (one LDS read and one
      // temper per lane); only words inside the look-ahead are used
      const uint32_t* wp = mt + mti + lane;
      const uint32_t w0 = temper(wp[0]);
      const uint32_t w1 = (uint32_t)wave_next((int)w0), w2 = (uint32_t)wave_next((int)w1),
                     w3 = (uint32_t)wave_next((int)w2), w4 = (uint32_t)wave_next((int)w3);
      (void)w3;
      // random() < 0.8 <=> N = (w0 >> 5) * 2^26 + (w1 >> 6) < lt08 <=> (w0 >> 5) * 2^32 + w1 <
      // lt08 * 64 (w1's low 6 bits cannot carry past a multiple of 64): one shift, one compare
      const uint64_t N64 = ((uint64_t)(w0 >> 5) << 32) | w1;
      // the decision at word t: [MASK] (2 words), else keep (random() < 0.5: w2's top bit clear,
      // 4 words), else a random word (randint's first word w4 accepted: 5 words; rejected: the
      // rare scan below); len 0 when the decision's words run past the look-ahead. Written as
      // selects on three compares and a shift, so that no lane-mask logic runs on the scalar unit.
      const bool mk = N64 < (lt08 << 6);
      const uint32_t top = w2 >> 31;  // 1: not keep
      const uint32_t r4 = w4 >> (32 - kV);
      const bool r4ok = r4 < (uint32_t)V;
      const int need = mk ? 2 : 4 + (int)top;
      int len = lane + need > kLook ? 0 : mk ? 2 : top ? (r4ok ? 5 : 0) : 4;
      int32_t tok = mk ? mask_id : top ? (int32_t)r4 : kKeep;
      if (!mk && top && !r4ok) {  // randint rejected its first word: scan on (rare)
        for (int j = 5; lane + j < kLook; ++j) {
          const uint32_t r = temper(wp[j]) >> (32 - kV);
          if (r < (uint32_t)V) {
            len = j + 1;
            tok = (int32_t)r;
            break;
          }
        }
      }
      // J_b[t] = start after 2^b decisions from t (64: stop, absorbing)
      int Jd[5];
      Jd[0] = len ? min(lane + len, 64) : 64;
#pragma unroll
      for (int b = 1; b < 5; ++b) {
        const int y = __shfl(Jd[b - 1], Jd[b - 1] & 63, 64);
        Jd[b] = Jd[b - 1] >= 64 ? 64 : y;
      }
      int p = 0;  // start of decision `lane` (lanes < 32)
#pragma unroll
      for (int b = 0; b < 5; ++b) {
        const int t = __shfl(Jd[b], p & 63, 64);
        if ((lane >> b) & 1) p = p >= 64 ? 64 : t;
      }
      const int lp = __shfl(len, p & 63, 64);
      const int32_t tp = __shfl(tok, p & 63, 64);
      // a prefix of the lanes (two compares, the scalar unit ANDs their ballots)
      const uint64_t okm = ballot(p < 64) & ballot(lp > 0) & 0xFFFFFFFFull;
      int take = __ffsll((unsigned long long)~okm) - 1;
      if (take > cnt - c) take = cnt - c;
      const int32_t tk = __shfl(tp, (lane - c) & 63, 64);  // decision k goes to lane c + k
      if (lane >= c && lane < c + take) res = tk;
      if (take > 0) {
        mti = uni(mti + (int)rdlane((uint32_t)p, take - 1) + (int)rdlane((uint32_t)lp, take - 1));
        c += take;
      } else {  // the first decision needs words past the look-ahead: draw it word by word
        wbase = -1024;
        wend = 0;
        int32_t t2;
        if (rand53() < lt08) t2 = mask_id;
        else if (below_half()) t2 = kKeep;
        else t2 = (int32_t)randint(0, V - 1);
        if (lane == c) res = t2;
        ++c;
      }
    }
    wbase = -1024;
    wend = 0;
    return res;
  }

  // random() = N / 2^53 with N = (w1 >> 5) * 2^26 + (w2 >> 6). `random() < p` is decided exactly
  // on N: N < ceil(p * 2^53) (see k_short / kLt08), so no floating point is needed.
  // two consecutive words with one window check when both are in the window
  __device__ void u32x2(uint32_t& a, uint32_t& b) {
    if (mti + 1 < wend) {
      a = rdlane(win, mti - wbase);
      b = rdlane(win, mti + 1 - wbase);
      mti = uni(mti + 2);
    } else {
      a = u32();
      b = u32();
    }
  }
  __device__ uint64_t rand53() {
    uint32_t a, b;
    u32x2(a, b);
    return ((uint64_t)(a >> 5) << 26) | (b >> 6);
  }
  __device__ bool below_half() {  // random() < 0.5  <=>  N < 2^52  <=>  w1 < 2^31
    uint32_t a, b;
    u32x2(a, b);
    return a < 0x80000000u;
  }
  __device__ uint32_t randbelow(uint32_t n) {
    const int k = 32 - __clz(n);
    uint32_t r = u32() >> (32 - k);
    while (r >= n) r = u32() >> (32 - k);
    return r;
  }
  __device__ int64_t randint(int64_t a, int64_t b) { return a + randbelow((uint32_t)(b - a + 1)); }
  __device__ int32_t randint32(int32_t a, int32_t b) { return a + (int32_t)randbelow((uint32_t)(b - a + 1)); }

};

// Token ids of the pair tables (the dense kept tokens, the sample tokens and labels): 2 bytes each
// when the vocab fits uint16 (lddl_ctx::id_bytes), else 4. The hot reader (gather_kernel) is
// templated on the type; the rare paths read through this runtime-width view.
struct IdPtr {
  void* p;
  int32_t ib;
  __device__ int32_t ld(int64_t i) const {
    return ib == 2 ? (int32_t)static_cast<const uint16_t*>(p)[i] : static_cast<const int32_t*>(p)[i];
  }
  __device__ void st(int64_t i, int32_t v) const {
    if (ib == 2) static_cast<uint16_t*>(p)[i] = (uint16_t)v;
    else static_cast<int32_t*>(p)[i] = v;
  }
};

struct PlanArgs {
  // kept corpus
  const int64_t* kscan;  // dense token offset of each kept sentence
  const int32_t* ks_len;
  const int64_t* kd_off;
  const int64_t* kp_off;
  const int64_t* ks_start;  // kept sentence k's pieces at ids[ks_start[k] ...]: the tokenizer's
  const int32_t* ids;       // layout (`dense` is filled by this launch's tail workgroups)
  IdPtr dense;              // out: kept tokens, packed (densify_group)
  int64_t n_kept_sent;
  int32_t n_part, n_dense_wg;  // workgroups >= n_part fill `dense`
  const int64_t* part_seed;
  // params
  int32_t seq, dup, masking, vocab_size, cls_id, sep_id, mask_id, max_pred;
  double short_seq_prob, ratio;
  uint64_t k_short;  // random() < short_seq_prob  <=>  N < k_short = ceil(short_seq_prob * 2^53)
  int32_t seq_r64;   // seq rounded up to a multiple of 64
  // outputs, slot base of partition p = dup * kd_off[kp_off[p]]
  PairDesc* desc;
  int32_t* jseq;       // per slot: j_i draws of the final partition shuffle
  SlotPool* spool;     // per slot (masking)
  int32_t* mtok;       // mask pool: slot s's decisions at 8 * moff8 .. + nmask (shuffled order)
  void* jpool;         // draw pool: j_i of random.shuffle(cand_indexes) at 16 * joff16 + i
  int32_t jbytes;      // 1 (target_seq_length <= 256: every j_i < 256) or 2 bytes per draw
  unsigned long long* pool_used;  // [0] masks, [1] overflow flag, [2] draws
  int64_t pool_cap, jpool_cap;
  int32_t* overflow;   // set when the pool is too small (the host re-plans with a larger one)
  int64_t* part_npairs;
  uint64_t* stamps;  // diagnostic build: [n_part][8]
  uint64_t* tl;      // diagnostic build: [n_part][2] s_memrealtime at start / end (100 MHz)
};

constexpr int kDocLds = 512;  // partitions with <= this many documents cache offsets in LDS
constexpr uint64_t kLt08 = 7205759403792794ull;  // ceil(0.8 (binary64) * 2^53): random() < 0.8

// Sentence lengths of one document through a 64-entry register window (lane l: sentence
// wbase + l) with their inclusive prefix sum, so a chunk end is one ballot and a span's length
// two readlanes. Lengths are < 2^24 (lddl_tokenize caps max_pieces), so 64 of them fit int32.
struct LenWin {
  const int32_t* len;  // ks_len + first kept sentence of the doc
  int n, wbase;
  int32_t win, pre;
  uint64_t fl;  // lanes whose sentence holds a literal [CLS]/[SEP]
  __device__ void reset(const int32_t* p, int nn) { len = p; n = nn; wbase = -1024; }
  // the first window of a document loaded ahead (issued one document early, so the chain does not
  // wait for it), then taken as the window at sentence 0
  int32_t pfw;
  __device__ void prefetch(const int32_t* p, int nn) {
    const int k = (int)threadIdx.x;
    pfw = k < nn ? p[k] : 0;
  }
  __device__ void reset_prefetched(const int32_t* p, int nn) {
    len = p;
    n = nn;
    wbase = 0;
    win = pfw;
    pre = wave_incl_scan(win & kLenMask);
    fl = ballot((win & kLenHasClsSep) != 0);
  }
  __device__ bool has(int j) const { return (unsigned)(j - wbase) < 64u; }  // (j >= 0)
  __device__ void load(int j) {
    wbase = j;
    const int k = j + (int)threadIdx.x;
    win = k < n ? len[k] : 0;
    pre = wave_incl_scan(win & kLenMask);
    fl = ballot((win & kLenHasClsSep) != 0);
  }
  __device__ int32_t at(int j) {  // raw length word (flags included)
    if (!has(j)) load(j);
    return (int32_t)rdlane((uint32_t)win, j - wbase);
  }
  // total length of sentences [a, b) (a < b); ORs their flags into `flags`
  __device__ int64_t sum(int a, int b, int32_t& flags) {
    if (!has(a)) load(a);
    if (!has(b - 1)) {  // longer than a window: sequential
      int64_t s = 0;
      for (int j = a; j < b; ++j) {
        const int32_t w = at(j);
        s += w & kLenMask;
        flags |= w;
      }
      return s;
    }
    const int32_t hi = (int32_t)rdlane((uint32_t)pre, b - 1 - wbase);
    const int32_t lo = a > wbase ? (int32_t)rdlane((uint32_t)pre, a - 1 - wbase) : 0;
    if (fl) {  // (a window without literal [CLS]/[SEP] skips the span mask: the common case)
      const int cnt = b - a;
      const uint64_t m = fl >> (a - wbase);
      if ((cnt >= 64 ? m : (m & ((1ull << cnt) - 1))) != 0) flags |= kLenHasClsSep;
    }
    return hi - lo;
  }
  // the smallest i in [a, lim) with length(a .. i) >= T, else lim - 1 (a < lim <= n): the end of
  // the reference's accumulate-until-target loops (pretrain.py:276-280, 314-317)
  __device__ int find(int a, int lim, int64_t T) {
    if (!has(a)) load(a);
    // (window sums are < 2^31: 32-bit compares; two ballots combined by one scalar AND)
    const int32_t T32 = T < -1 ? -1 : T > INT32_MAX ? INT32_MAX : (int32_t)T;
    for (int pass = 0; pass < 2; ++pass) {
      const int32_t base = a > wbase ? (int32_t)rdlane((uint32_t)pre, a - 1 - wbase) : 0;
      const int j = wbase + (int)threadIdx.x;
      const uint64_t m = ballot((uint32_t)(j - a) < (uint32_t)(lim - a)) & ballot(pre - base >= T32);
      if (m) return wbase + __ffsll((unsigned long long)m) - 1;
      if (wbase + 64 >= lim) return lim - 1;
      if (pass == 0 && wbase != a) load(a);  // restart the window at a and look again
      else break;
    }
    int64_t s = 0;  // more than 64 sentences: sequential
    for (int i = a;; ++i) {
      s += at(i) & kLenMask;
      if (i == lim - 1 || s >= T) return i;
    }
  }
};

// token j (0-based) of the span that starts at kept sentence k0 (slow path only: a literal
// [CLS]/[SEP] in the pair), read from the tokenizer's layout
__device__ int32_t span_token(const PlanArgs& A, int64_t k0, int64_t j) {
  const int64_t x = A.kscan[k0] + j;
  int64_t k = k0;
  while (A.kscan[k + 1] <= x) ++k;
  return A.ids[A.ks_start[k] + (x - A.kscan[k])];
}

// Kept tokens packed densely (see densify_kernel below):
// one wave: kept sentences [k0, k0 + 64)
__device__ inline void densify_group(int64_t k0, const int64_t* __restrict__ ks_start,
                                     const int32_t* __restrict__ ks_len,
                                     const int64_t* __restrict__ kscan, int64_t n,
                                     const int32_t* __restrict__ ids, IdPtr dense) {
  const int lane = threadIdx.x & 63;
  const int64_t k = k0 + lane;
  const bool ok = k < n;
  const int32_t len = ok ? ks_len[k] & kLenMask : 0;
  const int64_t st = ok ? ks_start[k] : 0;
  const int32_t incl = wave_incl_scan(len);
  const int32_t total = __builtin_amdgcn_readlane(incl, 63);  // (uniform: scalar loop bounds)
  const int64_t base = kscan[k0];
  // the sentence loop indices are wave-uniform: lane values via readlane, not LDS permutes
  auto rl = [](int32_t v, int i) { return __builtin_amdgcn_readlane(v, i); };
  // kU chunks of 64 tokens per round: their sources first, then all kU loads, then the stores,
  // so a wave has kU loads in flight instead of one dependent load -> store per chunk
  constexpr int kU = 4;  // (8: 6.0 -> 6.3 ms, profiles/r06y)
  int j = 0;
  for (int32_t c0 = 0; c0 < total; c0 += 64 * kU) {
    int64_t src[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int32_t cu = c0 + 64 * u, x = cu + lane, hi = min(cu + 63, total - 1);
      src[u] = 0;
      if (cu < total) {
        while (rl(incl, j) <= cu) ++j;  // first sentence overlapping the chunk
        for (int jj = j;; ++jj) {
          const int32_t e = rl(incl, jj);
          const int32_t b = e - rl(len, jj);
          const int64_t s = ((int64_t)rl((int32_t)(st >> 32), jj) << 32) | (uint32_t)rl((int32_t)st, jj);
          if (x >= b && x < e) src[u] = s + (x - b);
          if (e > hi) break;
        }
      }
    }
    int32_t v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) v[u] = c0 + 64 * u + lane < total ? ids[src[u]] : 0;
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (c0 + 64 * u + lane < total) dense.st(base + c0 + 64 * u + lane, v[u]);
  }
}

// waves per SIMD the compiler must keep: 8 caps the kernel at 78 SGPRs (140 spilled to VGPR
// lanes); 6 lets it use all 106 (59 spilled) at 7 waves/SIMD, 176 -> 169.6 ms per 10 GB
// (profiles/r02_plan_minw_ab.txt)
// kDocsLds: every partition's document offsets fit the LDS table (host-checked: <= kDocLds
// documents), so the document lookups carry no global-memory branch; kJB: bytes per shuffle draw
template <bool kDocsLds, int kJB>
__global__ void __launch_bounds__(64, 6) plan_replay_kernel(PlanArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* s_mt = reinterpret_cast<uint32_t*>(smem);
  int32_t* s_doc = reinterpret_cast<int32_t*>(s_mt + kN + kLook);  // [kDocLds + 1]
  const int p = blockIdx.x;
  const int lane = threadIdx.x;
  const bool leader = lane == 0;
  if (p >= A.n_part) {
    // Workgroups past the partitions pack `dense` (what densify_kernel would do after this
    // launch). Dispatched in order, they start as the last partitions' waves are placed and
    // run in the slots the planner's tail leaves idle (a separate launch before or beside the
    // planner delays its dispatch).
    for (int64_t g = p - A.n_part; g * 64 < A.n_kept_sent; g += A.n_dense_wg)
      densify_group(g * 64, A.ks_start, A.ks_len, A.kscan, A.n_kept_sent, A.ids, A.dense);
    return;
  }
#ifdef LDDL_STAMPS
  uint64_t st_acc[kStampRegions] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  [[maybe_unused]] uint64_t st_t = STAMP_T();
#ifdef LDDL_STAMPS
  const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
#endif
  WaveRng rng{s_mt, 0, 0, 0, 0u
#ifdef LDDL_STAMPS
              , 0, 0
#endif
  };
  rng.seed_i64(A.part_seed[p]);
  const int64_t d0 = A.kp_off[p];
  const int32_t nd = (int32_t)(A.kp_off[p + 1] - d0);  // (partition-local indices are 32-bit)
  const int64_t kbase = A.kd_off[d0];
  if (kDocsLds)
    for (int64_t d = lane; d <= nd; d += 64) s_doc[d] = (int32_t)(A.kd_off[d0 + d] - kbase);
  __syncthreads();
  auto doc_loc = [&](int32_t d) -> int32_t {  // first kept sentence of document d, partition-local
    if constexpr (kDocsLds) return uni(s_doc[d]);
    else return uni((int32_t)(A.kd_off[d0 + d] - kbase));
  };
  const int32_t* ks_len_p = A.ks_len + kbase;
  const int64_t base = (int64_t)A.dup * kbase;
  const int32_t max_num = A.seq - 3;
  // this wave's current chunks of the mask pool and of the shuffle-draw pool: next entry, entries
  // left (32-bit compares), and whether the chunk lies inside the pool
  int64_t pool_cur = 0, jpool_cur = 0;
  int32_t pool_left = 0, jpool_left = 0;
  bool pool_fits = true, jpool_fits = true;
  LenWin La, Lb;
  int64_t np = 0;
  constexpr int kPrioLevels = 4;  // priority levels used (s_setprio has 4)
  // issue priority by progress: a SIMD issues its highest-priority (then oldest) wave first, so
  // waves that are behind (e.g. a partition dispatched into a freed slot) catch up and the waves
  // of a SIMD finish together instead of leaving the last ones running alone
  int prio_q = -1;
  const int64_t prio_tot = (int64_t)A.dup * nd;
  // the priority steps at the document counts where progress crosses a quarter (no 64-bit
  // division per document)
  int32_t prio_next = 0, prio_done = 0;
  if (nd > 0) La.prefetch(ks_len_p + doc_loc(0), doc_loc(1) - doc_loc(0));
  for (int dp = 0; dp < A.dup; ++dp) {
    for (int32_t di = 0; di < nd; ++di) {
      if (prio_done >= prio_next) {
        ++prio_q;
        prio_next = (int32_t)(((int64_t)(prio_q + 1) * prio_tot + kPrioLevels - 1) / kPrioLevels);
        const int lvl = kPrioLevels - 1 - prio_q;
        if (lvl >= 3) __builtin_amdgcn_s_setprio(3);
        else if (lvl == 2) __builtin_amdgcn_s_setprio(2);
        else if (lvl == 1) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      }
      ++prio_done;
      const int32_t ls0 = doc_loc(di);
      const int64_t s0 = kbase + ls0;
      const int ns = doc_loc(di + 1) - ls0;
      // (the document's first length window was loaded one document ago; 1.5 ms per 10 GB,
      // profiles/r06p2_planner_loop_ab.txt)
      La.reset_prefetched(ks_len_p + ls0, ns);
      {
        const int32_t dn = di + 1 < nd ? di + 1 : 0;  // the next document (of this or the next pass)
        const int32_t nl0 = doc_loc(dn);
        La.prefetch(ks_len_p + nl0, doc_loc(dn + 1) - nl0);
      }
      int32_t target = max_num;
      if (rng.rand53() < A.k_short) target = rng.randint32(2, max_num);
      // chunks: sentences are accumulated until the target length or the document end
      // (pretrain.py:276-280); after a random-next pair the unused sentences are put back
      // (320-321), so the next chunk starts right after A
      for (int chunk0 = 0; chunk0 < ns;) {
        const int i = La.find(chunk0, ns, target);  // the chunk is [chunk0, i]
        const int chunk_n = i - chunk0 + 1;
        const int a_end = chunk_n >= 2 ? rng.randint32(1, chunk_n - 1) : 1;
        int32_t flags = 0;
        const int64_t la = La.sum(chunk0, chunk0 + a_end, flags);
        int64_t lb = 0, b_ks;
        int32_t rn = 0;
        int next0;
        STAMP_ADD(0, st_t);
        if (chunk_n == 1 || rng.below_half()) {
          rn = 1;
          const int64_t target_b = target - la;
          int32_t rd = 0;
          for (int t = 0; t < 10; ++t) {
            rd = rng.randint32(0, nd - 1);
            if (rd != di) break;
          }
          if (rd == di) rn = 0;
          const int32_t r0l = doc_loc(rd);
          const int rns = doc_loc(rd + 1) - r0l;
          const int rstart = rng.randint32(0, rns - 1);
          b_ks = kbase + (r0l + rstart);
          Lb.reset(ks_len_p + r0l, rns);
          const int jb = Lb.find(rstart, rns, target_b);  // B is [rstart, jb] (314-317)
          lb = Lb.sum(rstart, jb + 1, flags);
          next0 = chunk0 + a_end;
        } else {
          b_ks = s0 + chunk0 + a_end;
          lb = La.sum(chunk0 + a_end, i + 1, flags);
          next0 = i + 1;
        }
        STAMP_ADD(3, st_t);
        // _truncate_seq_pair
        int32_t a_front = 0, b_front = 0, na = (int32_t)la, nb = (int32_t)lb;
        rng.trunc_draws(na, nb, max_num, a_front, b_front);
        STAMP_ADD(5, st_t);
        const int64_t slot = base + np;
        // every lane stores the same record: the wave's identical writes merge into one, and no
        // exec-mask branch (3 scalar instructions + a branch) is spent on a leader-only store
        A.desc[slot] = PairDesc{s0 + chunk0, b_ks, a_front, na, b_front,
                                nb | (int32_t)((uint32_t)rn << 31)};
        if (A.masking) {
          // candidates = positions of [CLS] A [SEP] B [SEP] whose token is not [CLS]/[SEP]; only
          // their count matters here (fy_resolve_kernel recovers the positions)
          int32_t nc = na + nb;
          if (flags & kLenHasClsSep) {  // literal [CLS]/[SEP] inside A or B: inspect the tokens
            int32_t c = 0;
            for (int32_t t = 0; t < na + nb; ++t) {
              const int32_t tok = uni(t < na ? span_token(A, s0 + chunk0, a_front + t)
                                             : span_token(A, b_ks, b_front + (t - na)));
              c += tok != A.cls_id && tok != A.sep_id;
            }
            nc = uni(c);
          }
          STAMP_ADD(1, st_t);
          // num_to_predict = round(len(tokens) * masked_lm_ratio) (pretrain.py:197): binary64
          // product, round half to even - the IEEE operations Python performs
          int32_t num = uni((int32_t)__builtin_rint((double)(na + nb + 3) * A.ratio));
          if (num < 1) num = 1;
          if (num > nc) num = nc;
          // pool space for this pair's shuffle draws (nc) and masks (num): bump allocation in
          // per-wave chunks (one atomic per kPoolChunk entries); each slot records its offsets
          if (num > pool_left) {
            const int32_t sz = num > kPoolChunk ? (num + 7) & ~7 : (int32_t)kPoolChunk;
            int64_t nb0 = 0;
            if (leader) nb0 = (int64_t)atomicAdd(&A.pool_used[0], (unsigned long long)sz);
            nb0 = ((int64_t)uni((int)(nb0 >> 32)) << 32) | (uint32_t)uni((int)(uint32_t)nb0);  // lane 0's
            pool_cur = nb0;
            pool_left = sz;
            pool_fits = nb0 + sz <= A.pool_cap;
          }
          if (nc > jpool_left) {
            const int32_t sz = nc > kPoolChunk ? (nc + 15) & ~15 : (int32_t)kPoolChunk;
            int64_t nb0 = 0;
            if (leader) nb0 = (int64_t)atomicAdd(&A.pool_used[2], (unsigned long long)sz);
            nb0 = ((int64_t)uni((int)(nb0 >> 32)) << 32) | (uint32_t)uni((int)(uint32_t)nb0);
            jpool_cur = nb0;
            jpool_left = sz;
            jpool_fits = nb0 + sz <= A.jpool_cap;
          }
          const int64_t mb = pool_cur, jb = jpool_cur;
          // 16-byte aligned regions (fy_resolve_kernel's uint4 I/O; 1-byte draws too); chunk sizes
          // are multiples of the steps, so num <= left implies step <= left
          pool_cur += (num + 7) & ~7;
          pool_left -= (num + 7) & ~7;
          jpool_cur += (nc + 15) & ~15;
          jpool_left -= (nc + 15) & ~15;
          const bool fits = pool_fits && jpool_fits;
          if (!fits) *A.overflow = 1;  // (uniform; every lane stores the same flag)
          // random.shuffle(cand_indexes): draws j_i (i = nc-1 .. 1) to the pool
          // The region's tail [nc, nc rounded up to 16) gets j_i = i: fy_resolve's steps there move
          // an entry onto itself, so its step loop needs no per-step guard. (Entry 0 is not
          // written here: fy_draws' lanes store their rejected words there, and fy_resolve
          // takes j_0 = 0 itself.)
          const int32_t ip = nc + lane;
          if constexpr (kJB == 1) {
            uint8_t* jd = static_cast<uint8_t*>(A.jpool) + jb;
            rng.fy_draws(nc, [&](int32_t i, uint32_t j) {
              if (fits) jd[i] = (uint8_t)j;  // (fits is uniform: a scalar branch)
            });
            if (fits && ip < ((nc + 15) & ~15)) jd[ip] = (uint8_t)ip;
          } else {
            uint16_t* jd = static_cast<uint16_t*>(A.jpool) + jb;
            rng.fy_draws(nc, [&](int32_t i, uint32_t j) {
              if (fits) jd[i] = (uint16_t)j;
            });
            if (fits && ip < ((nc + 15) & ~15)) jd[ip] = (uint16_t)ip;
          }
          STAMP_ADD(2, st_t);
          // decisions of the masked candidates in shuffled order (pretrain.py:208-221)
          for (int32_t c0 = 0; c0 < num; c0 += 64) {
            const int cmax = min(64, num - c0);
            const int32_t mytok = rng.mask_decisions(cmax, kLt08, A.vocab_size, A.mask_id);
            if (fits && lane < cmax) A.mtok[mb + c0 + lane] = mytok;
          }
          STAMP_ADD(4, st_t);
          // (all lanes, as the descriptor above)
          A.spool[slot] = SlotPool{(uint32_t)(mb >> 3), (uint32_t)(jb >> 4), num, nc};
        }
        ++np;
        chunk0 = next0;
      }
    }
  }
  // random.shuffle(partition_pairs) (pretrain.py:401): record the draws j_i, i = np-1 .. 1
  // (64 at a time through writelane); shuffle_sort_kernel resolves the swaps.
  STAMP_ADD(0, st_t);
  {
    int32_t* js = A.jseq + base;
    rng.fy_draws(np, [&](int32_t i, uint32_t j) { js[i] = (int32_t)j; });  // (js[0] is never read)
  }
  STAMP_ADD(6, st_t);
#ifdef LDDL_STAMPS
  st_acc[7] = rng.n_pass * 1000000 / (rng.n_win ? rng.n_win : 1);  // passes per window x 1e6
  if (leader && A.stamps)
    for (int r = 0; r < kStampRegions; ++r) A.stamps[(int64_t)p * kStampRegions + r] = st_acc[r];
  if (leader && A.tl) {
    A.tl[2 * (int64_t)p] = rt0;
    A.tl[2 * (int64_t)p + 1] = __builtin_amdgcn_s_memrealtime();
  }
#endif
  if (leader) A.part_npairs[p] = np;
}

// ---------------------------------------------------------------------------------------------
// Native RNG mode (LDDL_RNG_NATIVE): the same algorithms (create_pairs_from_document,
// _truncate_seq_pair, create_masked_lm_predictions, the partition shuffle) drawing from
// Philox4x32-10 instead of one sequential MT19937 per partition, so every (duplicate, document)
// walk and every pair's masking runs in its own lane. A stream is keyed by
// (native_seed, part_seed[p]) and counted by the unit's or pair's index inside its partition, so
// a partition's output does not depend on how partitions are batched or sharded.
// Distributions are those of the reference: in the walk, randint / _randbelow by the same
// bit-length rejection and random() < p on the same 53-bit integer, each truncation side a fair
// coin; in the masking, the masked set a uniform num_to_predict-subset of the candidates (Floyd's
// algorithm: the shuffled prefix of pretrain.py:197-207 is a uniform subset) and 80/10/10
// decisions per masked token, both from one 32-bit draw each (exact uniform integers by Lemire's
// multiply-shift with rejection).
// ---------------------------------------------------------------------------------------------
__device__ inline uint64_t mix64(uint64_t x) {  // splitmix64 finaliser
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ inline uint64_t part_key(uint64_t native_seed, int64_t part_seed) {
  return mix64(native_seed ^ mix64((uint64_t)part_seed + 0x9E3779B97F4A7C15ull));
}

enum : uint32_t { kStreamWalk = 1, kStreamMask = 2, kStreamOrder = 3, kStreamDecide = 4 };

struct CtrRng {
  uint2 key;
  uint32_t id0, id1, blk;
  uint4 buf;
  int have;
  __device__ CtrRng(uint64_t k, int64_t index, uint32_t stream)
      : key{(uint32_t)k, (uint32_t)(k >> 32)},
        id0((uint32_t)index),
        id1((uint32_t)((uint64_t)index >> 32) << 4 | stream),
        blk(0),
        have(0) {}
  __device__ uint32_t u32() {
    if (have == 0) {
      buf = Philox::gen(make_uint4(blk++, id0, id1, 0x6C64646Cu), key);
      have = 4;
    }
    --have;
    return have == 3 ? buf.x : have == 2 ? buf.y : have == 1 ? buf.z : buf.w;
  }
  __device__ uint64_t rand53() {  // the 53-bit integer behind random()
    const uint32_t a = u32() >> 5, b = u32() >> 6;
    return ((uint64_t)a << 26) | b;
  }
  __device__ bool coin() { return u32() < 0x80000000u; }
  __device__ uint32_t randbelow(uint32_t n) {  // _randbelow: k-bit draws until < n
    const int k = 32 - __clz(n);
    uint32_t r = u32() >> (32 - k);
    while (r >= n) r = u32() >> (32 - k);
    return r;
  }
  __device__ int64_t randint(int64_t a, int64_t b) { return a + randbelow((uint32_t)(b - a + 1)); }
  __device__ int32_t heads(int32_t n) {  // number of heads in n fair coins
    int32_t h = 0;
    for (; n >= 32; n -= 32) h += __popc(u32());
    if (n > 0) h += __popc(u32() & ((1u << n) - 1u));
    return h;
  }
};

struct NativeArgs {
  const int32_t* ks_len;
  const int64_t* kd_off;
  const int64_t* kp_off;
  const int64_t* kscan;
  IdPtr dense;
  const int64_t* part_seed;
  int64_t n_part, n_units, unit0;  // units dup * (kp_off[0] .. kp_off[n_part])
  uint64_t native_seed, k_short;
  int32_t seq, dup, masking, cls_id, sep_id, mask_id, vocab_size;
  double ratio;
  int64_t* ucnt;        // count pass: pairs of each (duplicate, document) unit
  const int64_t* uoff;  // emit pass: first pair of each unit (exclusive scan of ucnt)
  const int64_t* part_base;
  PairDesc* desc;
  int32_t* nmask;
  int32_t* ncand;
  int32_t* ppart;
  const int64_t* moff;
  uint16_t* mpos;
  int32_t* mtok;
  int64_t* src;
  int64_t n_pairs;
  int32_t words;  // bitmap words per lane (mask kernel)
};

// token t of the window [front, front + n) of the span starting at kept sentence k
__device__ inline int32_t win_token(const NativeArgs& A, int64_t k, int32_t front, int32_t t) {
  return A.dense.ld(A.kscan[k] + front + t);
}

// One partition's walk tables: cumulative kept-sentence lengths and document starts, both
// partition-relative. Staged in LDS when the partition fits (every length sum and search of the
// walk is then an LDS read), else read from the global prefix `g_pre` (int64 over all kept
// sentences) and kd_off. The branch is uniform over the workgroup.
struct WalkTab {
  const int32_t* s_pre;  // [nsp + 1]
  const int32_t* s_doc;  // [nd + 1]
  const int64_t* g_pre;
  const int64_t* g_doc;  // kd_off + d0
  int64_t sb, pre_sb;    // the partition's first kept sentence, g_pre[sb]
  bool lds;
  __device__ int64_t pre(int64_t i) const { return lds ? (int64_t)s_pre[i] : g_pre[sb + i] - pre_sb; }
  __device__ int32_t doc(int64_t d) const { return lds ? s_doc[d] : (int32_t)(g_doc[d] - sb); }
};

// Smallest e in [i, end) whose sentences i..e reach `need` = pre(i) + target (pre(e + 1) >= need),
// else end - 1: the chunk / random-B loops of create_pairs_from_document (pretrain.py:276-280,
// 300-304) as a galloping search over the cumulative lengths (pre(i) < need on entry).
__device__ inline int32_t first_reaching(const WalkTab& W, int32_t i, int32_t end, int64_t need) {
  int32_t a = i, b = i + 1;
  for (int32_t step = 1;; step <<= 1) {
    b = a + step;
    if (b >= end) {
      b = end;
      break;
    }
    if (W.pre(b) >= need) break;
    a = b;
  }
  if (b == end && W.pre(end) < need) return end - 1;
  while (b - a > 1) {  // pre(a) < need <= pre(b)
    const int32_t m = (a + b) >> 1;
    if (W.pre(m) >= need) b = m;
    else a = m;
  }
  return b - 1;
}

// Literal [CLS]/[SEP] among kept sentences [x, y) of the partition (rare: only partitions that
// hold one at all look).
__device__ inline int32_t range_flags(const NativeArgs& A, bool has_flags, int64_t sb, int32_t x,
                                      int32_t y) {
  int32_t f = 0;
  if (has_flags)
    for (int32_t j = x; j < y; ++j) f |= A.ks_len[sb + j];
  return f & kLenHasClsSep;
}

constexpr int kNativeThreads = 256;

// Unit r = (duplicate dp, document dl) of partition p is r = dp * nd + dl (the reference's
// `for _ in range(dup): for doc in docs` order); its global index is dup * (kp_off[p] -
// kp_off[0]) + r. One workgroup per partition: the partition's cumulative sentence lengths and
// document starts are staged in LDS, then every lane walks units, one chunk (pair) per loop
// iteration, taking the partition's next unit from an LDS counter when its unit ends - so a lane
// whose document is short does not idle while another lane's runs on. Chunk ends, A/B lengths and
// the random-next B span are LDS searches over the cumulative lengths (no per-sentence loop).
// EMIT = false counts each unit's pairs; EMIT = true replays the identical draws and writes them
// at uoff[unit].
template <bool EMIT>
__global__ void __launch_bounds__(kNativeThreads) plan_native_kernel(NativeArgs A, const int64_t* g_pre,
                                                                     int32_t lds_words) {
  extern __shared__ int32_t s_tab[];
  __shared__ int32_t s_next;
  const int64_t p = blockIdx.x;
  const int64_t d0 = A.kp_off[p], nd = A.kp_off[p + 1] - d0;
  const int64_t sb = A.kd_off[d0], nsp = A.kd_off[d0 + nd] - sb;
  WalkTab W{s_tab, s_tab + nsp + 1, g_pre, A.kd_off + d0, sb, 0,
            nsp + nd + 2 <= (int64_t)lds_words};
  bool flag_any = false;
  if (W.lds) {
    int32_t* pre = s_tab;
    int32_t* dst = s_tab + nsp + 1;
    for (int64_t i = threadIdx.x; i < nsp; i += kNativeThreads) {
      const int32_t v = A.ks_len[sb + i];
      pre[i + 1] = v & kLenMask;
      flag_any |= (v & kLenHasClsSep) != 0;
    }
    for (int64_t d = threadIdx.x; d <= nd; d += kNativeThreads) dst[d] = (int32_t)(A.kd_off[d0 + d] - sb);
    if (threadIdx.x == 0) {
      pre[0] = 0;
      s_next = kNativeThreads;
    }
    __syncthreads();
    // in-place inclusive scan of pre[1 .. nsp]: a contiguous run per thread, then the runs' sums
    const int32_t per = (int32_t)((nsp + kNativeThreads - 1) / kNativeThreads);
    const int32_t x0 = 1 + (int32_t)threadIdx.x * per;
    const int32_t x1 = min(x0 + per, (int32_t)nsp + 1);
    int32_t run = 0;
    for (int32_t x = x0; x < x1; ++x) run += pre[x];
    __shared__ int32_t s_wsum[kNativeThreads / 64];
    const int32_t inc = wave_incl_scan(run);
    if ((threadIdx.x & 63) == 63) s_wsum[threadIdx.x >> 6] = inc;
    __syncthreads();
    int32_t off = inc - run;
    for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) off += s_wsum[w];
    for (int32_t x = x0; x < x1; ++x) {
      off += pre[x];
      pre[x] = off;
    }
  } else {
    W.pre_sb = g_pre[sb];
    for (int64_t i = threadIdx.x; i < nsp; i += kNativeThreads)
      flag_any |= (A.ks_len[sb + i] & kLenHasClsSep) != 0;
    if (threadIdx.x == 0) s_next = kNativeThreads;
  }
  const bool has_flags = __syncthreads_or(flag_any) != 0;
  const int64_t nu = (int64_t)A.dup * nd;
  const int64_t ug0 = (int64_t)A.dup * (d0 - A.kp_off[0]);  // global index of the partition's unit 0
  const uint64_t key = part_key(A.native_seed, A.part_seed[p]);
  const int32_t max_num = A.seq - 3;
  int64_t r = threadIdx.x;
  bool fresh = true;
  CtrRng rng(key, 0, kStreamWalk);
  int32_t s0 = 0, ns = 0, i = 0, target = 0, dl = 0;
  int64_t np = 0, base = 0;
  while (__builtin_amdgcn_ballot_w64(r < nu)) {
    if (r < nu) {
      if (fresh) {  // a new unit: its document and target length (pretrain.py:259-262)
        fresh = false;
        dl = (int32_t)(r % nd);
        rng = CtrRng(key, r, kStreamWalk);
        s0 = W.doc(dl);
        ns = W.doc(dl + 1) - s0;
        i = 0;
        np = 0;
        if (EMIT) base = A.uoff[ug0 + r];
        target = max_num;
        if (rng.rand53() < A.k_short) target = (int32_t)rng.randint(2, max_num);
      }
      if (i < ns) {  // one chunk -> one pair
        const int64_t c_pre = W.pre(s0 + i);
        const int32_t e = first_reaching(W, s0 + i, s0 + ns, c_pre + target) - s0;
        const int32_t chunk0 = i, chunk_n = e - i + 1;
        const int32_t a_end = chunk_n >= 2 ? (int32_t)rng.randint(1, chunk_n - 1) : 1;
        const int64_t la = W.pre(s0 + chunk0 + a_end) - c_pre;
        int64_t lb, b_ks;
        int32_t rn = 0, flags = 0;
        if (chunk_n == 1 || rng.coin()) {  // random next (pretrain.py:291-321)
          rn = 1;
          const int64_t target_b = target - la;
          int64_t rd = 0;
          for (int t = 0; t < 10; ++t) {
            rd = rng.randint(0, nd - 1);
            if (rd != dl) break;
          }
          if (rd == dl) rn = 0;
          const int32_t r0 = W.doc(rd), rns = W.doc(rd + 1) - r0;
          const int32_t rstart = (int32_t)rng.randint(0, rns - 1);
          const int64_t b_pre = W.pre(r0 + rstart);
          const int32_t be = first_reaching(W, r0 + rstart, r0 + rns, b_pre + target_b);
          lb = W.pre(be + 1) - b_pre;
          b_ks = sb + r0 + rstart;
          if (EMIT && A.masking)
            flags = range_flags(A, has_flags, sb, s0 + chunk0, s0 + chunk0 + a_end) |
                    range_flags(A, has_flags, sb, r0 + rstart, be + 1);
          i = chunk0 + a_end;  // the unused segments are put back (pretrain.py:320-321)
        } else {
          lb = W.pre(s0 + e + 1) - W.pre(s0 + chunk0 + a_end);
          b_ks = sb + s0 + chunk0 + a_end;
          if (EMIT && A.masking) flags = range_flags(A, has_flags, sb, s0 + chunk0, s0 + e + 1);
          i = e + 1;
        }
        // _truncate_seq_pair: which side each trim hits is fixed (see WaveRng::trunc_draws); front
        // or back is a fair coin per trim
        int32_t na = (int32_t)la, nb = (int32_t)lb, a_front = 0, b_front = 0;
        const int32_t T = na + nb - max_num;
        if (T > 0) {
          const int32_t dd = na - nb, ad = dd < 0 ? -dd : dd;
          const int32_t nA = (dd > 0 ? min(dd, T) : 0) + (T > ad ? (T - ad) / 2 : 0);
          a_front = rng.heads(nA);
          b_front = rng.heads(T - nA);
          na -= nA;
          nb -= T - nA;
        }
        if (EMIT) {
          const int64_t q = base + np;
          const int64_t a_ks = sb + s0 + chunk0;
          A.desc[q] = PairDesc{a_ks, b_ks, a_front, na, b_front, nb | (int32_t)((uint32_t)rn << 31)};
          A.ppart[q] = (int32_t)p;
          if (A.masking) {
            int32_t nc = na + nb;
            if (flags) {  // literal [CLS]/[SEP] in the text are not candidates
              nc = 0;
              for (int32_t t = 0; t < na + nb; ++t) {
                const int32_t tok = t < na ? win_token(A, a_ks, a_front, t)
                                           : win_token(A, b_ks, b_front, t - na);
                nc += tok != A.cls_id && tok != A.sep_id;
              }
            }
            int32_t num = (int32_t)rint((double)(na + nb + 3) * A.ratio);
            if (num < 1) num = 1;
            if (num > nc) num = nc;
            A.nmask[q] = num;
            A.ncand[q] = nc;
          }
        }
        ++np;
      }
      if (i >= ns) {  // the unit is done: take the partition's next one
        if (!EMIT) A.ucnt[ug0 + r] = np;
        r = atomicAdd(&s_next, 1);
        fresh = true;
      }
    }
  }
}

// LDS words one partition's walk tables take; the largest over all partitions
__global__ void native_part_need_kernel(const int64_t* kp_off, const int64_t* kd_off, int64_t n_part,
                                        unsigned long long* need_max) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_part) return;
  const int64_t d0 = kp_off[p], d1 = kp_off[p + 1];
  atomicMax(need_max, (unsigned long long)(kd_off[d1] - kd_off[d0] + (d1 - d0) + 2));
}

struct KeptLenOnly {
  const int32_t* v;
  __device__ int64_t operator()(int64_t i) const { return v[i] & kLenMask; }
};

__global__ void native_part_base_kernel(const int64_t* kp_off, int64_t n_part, int32_t dup,
                                        const int64_t* uoff, int64_t* part_base) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p <= n_part) part_base[p] = uoff[(int64_t)dup * (kp_off[p] - kp_off[0])];
}

// Uniform integer in [0, n) from a 32-bit draw: Lemire's multiply-shift with the exact rejection
// (taken with probability < n / 2^32, so the lanes of a wave stay in step).
__device__ inline uint32_t lemire_below(uint32_t x, uint32_t n, CtrRng& rng) {
  uint64_t m = (uint64_t)x * n;
  if ((uint32_t)m < n) {
    const uint32_t t = (0u - n) % n;
    while ((uint32_t)m < t) m = (uint64_t)rng.u32() * n;
  }
  return (uint32_t)(m >> 32);
}

// 80 / 10 / 10 of create_masked_lm_predictions (pretrain.py:214-229) on one 32-bit draw:
// [MASK] below ceil(0.8 * 2^32), the original token below ceil(0.9 * 2^32), else a random token.
constexpr uint32_t kNat80 = 3435973837u, kNat90 = 3865470567u;

// Masked positions of 64 consecutive pairs per wave (one lane per pair), in lock step so that
// every lane's Philox refill comes at the same iteration:
//  1. Floyd's sampling of num candidate indices out of nc (a uniform num-subset: the shuffled
//     prefix of pretrain.py:197-207), one draw per step, into a lane-private LDS bitmap;
//  2. the set bits in ascending order (= sorted(masked_lms, key=index)), each with an 80/10/10
//     decision from its own stream (two draws per mask, whatever the decision), staged in LDS;
//  3. the wave's masks are one contiguous run of the pool (moff is the planner-order scan), copied
//     out with coalesced stores.
// Every draw's stream position depends on the pair alone (the sampling and the decisions use
// separate streams), so a pair's masks do not depend on the pairs that share its wave.
__global__ void __launch_bounds__(256) mask_native_kernel(NativeArgs A, int32_t stage_cap) {
  extern __shared__ __attribute__((aligned(16))) uint8_t s_mn[];
  const int w = wave_id(), lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  const int64_t q0 = ((int64_t)blockIdx.x * nw + w) * 64;
  if (q0 >= A.n_pairs) return;
  uint32_t* bm = reinterpret_cast<uint32_t*>(s_mn) + (size_t)w * A.words * 64 + lane;
  int32_t* stok = reinterpret_cast<int32_t*>(s_mn + (size_t)nw * A.words * 64 * 4) + (size_t)w * stage_cap;
  uint16_t* spos = reinterpret_cast<uint16_t*>(s_mn + (size_t)nw * A.words * 64 * 4 +
                                                (size_t)nw * stage_cap * 4) + (size_t)w * stage_cap;
  const int64_t q = q0 + lane;
  const bool valid = q < A.n_pairs;
  const int64_t qv = valid ? q : q0;
  const int64_t qe = q0 + 64 < A.n_pairs ? q0 + 64 : A.n_pairs;
  const int64_t m0 = A.moff[q0];
  const int32_t mend = (int32_t)(A.moff[qe] - m0);
  const int32_t num = valid ? A.nmask[qv] : 0;
  const int32_t nc = A.ncand[qv];
  const int32_t mb = (int32_t)(A.moff[qv] - m0);
  const PairDesc d = A.desc[qv];
  const int32_t na = d.na, nb = d.nb_rn & 0x7FFFFFFF;
  const int64_t p = A.ppart[qv];
  const uint64_t key = part_key(A.native_seed, A.part_seed[p]);
  const int64_t idx = qv - A.part_base[p];
  for (int i = 0; i < A.words; ++i) bm[i * 64] = 0u;
  CtrRng rng(key, idx, kStreamMask);
  for (int32_t s = 0; __builtin_amdgcn_ballot_w64(s < num); ++s) {
    const uint32_t u = rng.u32();
    if (s < num) {
      const uint32_t j = (uint32_t)(nc - num + s);
      const uint32_t t = lemire_below(u, j + 1u, rng);
      const uint32_t wt = bm[(t >> 5) * 64];
      const uint32_t pick = (wt >> (t & 31)) & 1u ? j : t;
      bm[(pick >> 5) * 64] |= 1u << (pick & 31);
    }
  }
  CtrRng drng(key, idx, kStreamDecide);
  const bool fast = nc == na + nb;
  int32_t wi = 0, tcur = 0, ccur = 0;  // bitmap word; slow path: token / candidate cursor
  uint32_t bits = num > 0 ? bm[0] : 0u;
  for (int32_t m = 0; __builtin_amdgcn_ballot_w64(m < num); ++m) {
    const uint32_t x = drng.u32(), y = drng.u32();
    if (m < num) {
      while (bits == 0u) bits = bm[++wi * 64];
      const int32_t ci = wi * 32 + __ffs(bits) - 1;
      bits &= bits - 1u;
      int32_t t = ci;
      if (!fast) {  // walk to the ci-th non-[CLS]/[SEP] token
        while (true) {
          const int32_t tok = tcur < na ? win_token(A, d.a_ks, d.a_front, tcur)
                                        : win_token(A, d.b_ks, d.b_front, tcur - na);
          if (tok != A.cls_id && tok != A.sep_id) {
            if (ccur == ci) break;
            ++ccur;
          }
          ++tcur;
        }
        t = tcur++;
        ++ccur;
      }
      const int32_t tok = x < kNat80 ? A.mask_id
                          : x < kNat90 ? kKeep
                                       : (int32_t)lemire_below(y, (uint32_t)A.vocab_size, drng);
      spos[mb + m] = (uint16_t)(t < na ? t + 1 : t + 2);
      stok[mb + m] = tok;
    }
  }
  wave_sync();
  for (int32_t i = lane; i < mend; i += 64) {
    A.mpos[m0 + i] = spos[i];
    A.mtok[m0 + i] = stok[i];
  }
}

// random.shuffle(partition_pairs), native: output row k of partition p takes pair perm_p(k), a
// keyed 4-round Feistel bijection on [0, 4^h) >= np restricted to [0, np) by cycle walking.
__global__ void __launch_bounds__(256) order_native_kernel(NativeArgs A) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= A.n_pairs) return;
  const int64_t p = A.ppart[q];
  const int64_t pb = A.part_base[p], np = A.part_base[p + 1] - pb;
  const uint64_t key = mix64(part_key(A.native_seed, A.part_seed[p]) ^ kStreamOrder);
  int bits = 1;
  while ((1ll << bits) < np) ++bits;
  const int h = (bits + 1) >> 1;
  const uint64_t hm = (1ull << h) - 1;
  uint64_t x = (uint64_t)(q - pb);
  do {
    uint64_t L = x >> h, R = x & hm;
    for (uint64_t rd = 0; rd < 4; ++rd) {
      const uint64_t f = mix64(R ^ key ^ (rd << 56)) & hm;
      const uint64_t nl = R;
      R = L ^ f;
      L = nl;
    }
    x = (L << h) | R;
  } while (x >= (uint64_t)np);
  A.src[q] = pb + (int64_t)x;
}


// The final per-partition Fisher-Yates swaps (draws from plan_replay_kernel) for partitions too
// large for shuffle_sort_kernel's LDS tables (more than min_np pairs): one lane swaps in global
// memory.

__global__ void __launch_bounds__(64) apply_shuffle_kernel(const int64_t* kd_off, const int64_t* kp_off,
                                                          int32_t dup, const int64_t* part_npairs,
                                                          const int32_t* jseq, int32_t* order,
                                                          int64_t min_np) {
  const int p = blockIdx.x;
  const int64_t base = (int64_t)dup * kd_off[kp_off[p]];
  const int64_t np = part_npairs[p];
  if (np <= min_np) return;  // (shuffle_sort_kernel's)
  const int32_t* js = jseq + base;
  int32_t* ord = order + base;
  for (int64_t k = threadIdx.x; k < np; k += 64) ord[k] = (int32_t)k;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int64_t i = np - 1; i > 0; --i) {
      const int32_t j = js[i];
      const int32_t t = ord[i];
      ord[i] = ord[j];
      ord[j] = t;
    }
  }
}

// The same permutation with no sequential chain at all (one workgroup of 1024 per partition of at
// most `cap` pairs; larger ones go to apply_shuffle_kernel). The backward Fisher-Yates
// x[i] <-> x[j_i], i = n-1 .. 1, on x = identity leaves, with succ(i) = the next step k > i that
// drew the same j (j_k = j_i) and first(v) = the first step that drew v:
//   x[i] = succ(i) ? R(succ(i)) : j_i  (i >= 1),   x[0] = first(0) ? R(first(0)) : 0,
// where R(k) follows f(k) = (j_k == k ? succ(k) : first(k)) to the end of its chain (the value
// step k moved out of position k is the one the last earlier-executed step wrote there, and so
// on). succ and first come from a bucket sort of the steps by their draw (LDS counters, a block
// scan, a scatter, then each bucket - a few steps on average - sorted by step), R from pointer
// jumping, everything over 1024 threads. LDS: three 16-bit arrays of n (the draws are read from
// global memory once, coalesced, into the one that later holds f and R).
__device__ inline uint32_t lds_add16(uint32_t* words, uint32_t v) {  // 16-bit counters, packed
  const uint32_t sh = 16u * (v & 1u);
  return (atomicAdd(&words[v >> 1], 1u << sh) >> sh) & 0xFFFFu;
}

constexpr int kShufThreads = 1024;  // one block per CU (its LDS): 16 waves hide the latencies
// The pair maps of map_pairs_kernel, written by the partition shuffle's last pass (any may be
// null): src[q] the slot of output pair q, slots[i] the i-th slot in planner order, dstq[i] the
// output position of the i-th pair in planner order; part_base[p] = the partition's first pair.
struct PairMaps {
  const int64_t* part_base;
  int64_t *src, *slots, *dstq;
};

__global__ void __launch_bounds__(kShufThreads) shuffle_sort_kernel(const int64_t* kd_off, const int64_t* kp_off,
                                                          int32_t dup, const int64_t* part_npairs,
                                                          const int32_t* __restrict__ jseq,
                                                          int32_t* __restrict__ order, int32_t cap,
                                                          PairMaps M) {
  extern __shared__ __attribute__((aligned(16))) uint8_t ss_smem[];
  const int p = blockIdx.x;
  const int32_t n = (int32_t)part_npairs[p];
  if (n > cap) return;  // (apply_shuffle_kernel's)
  const int32_t capw = (cap + 2) & ~1;
  uint32_t* cntw = reinterpret_cast<uint32_t*>(ss_smem);        // bucket counters -> ends
  uint16_t* cnt = reinterpret_cast<uint16_t*>(ss_smem);
  uint16_t* srt = reinterpret_cast<uint16_t*>(ss_smem) + capw;  // steps by bucket
  uint16_t* r = srt + capw;                                     // j, then f, then R
  const int64_t base = (int64_t)dup * kd_off[kp_off[p]];
  const int32_t* __restrict__ js = jseq + base;
  // succ(i) (or ~j_i when step i is the last to draw j_i), then the permutation
  int32_t* __restrict__ ord = order + base;
  const int tid = threadIdx.x;
  for (int32_t w = tid; w < capw / 2; w += kShufThreads) cntw[w] = 0u;
  for (int32_t i = tid; i < n; i += kShufThreads) r[i] = (uint16_t)js[i];
  __syncthreads();
  for (int32_t i = 1 + tid; i < n; i += kShufThreads) (void)lds_add16(cntw, r[i]);
  __syncthreads();
  {  // exclusive scan of the counts: a run per thread, then the runs' sums
    __shared__ int32_t s_w[kShufThreads / 64];
    const int32_t per = (n + kShufThreads - 1) / kShufThreads;
    const int32_t x0 = tid * per, x1 = min(x0 + per, n);
    int32_t run = 0;
    for (int32_t x = x0; x < x1; ++x) run += cnt[x];
    const int32_t inc = wave_incl_scan(run);
    if ((tid & 63) == 63) s_w[tid >> 6] = inc;
    __syncthreads();
    int32_t off = inc - run;
    for (int w = 0; w < (tid >> 6); ++w) off += s_w[w];
    for (int32_t x = x0; x < x1; ++x) {
      const int32_t c = cnt[x];
      cnt[x] = (uint16_t)off;
      off += c;
    }
  }
  __syncthreads();
  for (int32_t i = 1 + tid; i < n; i += kShufThreads) srt[lds_add16(cntw, r[i])] = (uint16_t)i;
  __syncthreads();  // cnt[v] = the end of bucket v now
  // each bucket sorted by step (insertion sort: a few entries), succ along it
  for (int32_t v = tid; v < n; v += kShufThreads) {
    const int32_t lo = v ? cnt[v - 1] : 0, hi = cnt[v];
    for (int32_t m = lo + 1; m < hi; ++m) {
      const uint16_t e = srt[m];
      int32_t y = m - 1;
      while (y >= lo && srt[y] > e) {
        srt[y + 1] = srt[y];
        --y;
      }
      srt[y + 1] = e;
    }
    for (int32_t m = lo; m < hi; ++m) ord[srt[m]] = m + 1 < hi ? (int32_t)srt[m + 1] : ~v;
  }
  __syncthreads();
  // f(k) = j_k == k ? succ(k) : first(k); R(k) = k at a chain's end (each thread reads the
  // draws it overwrites)
  for (int32_t k = tid; k < n; k += kShufThreads) {
    int32_t f = -1;
    if (k > 0) {
      if (r[k] == k) {
        f = ord[k];
      } else {
        const int32_t lo = cnt[k - 1], hi = cnt[k];
        f = lo < hi ? (int32_t)srt[lo] : -1;
      }
    }
    r[k] = (uint16_t)(f < 0 ? k : f);
  }
  __syncthreads();
  for (;;) {  // pointer jumping: R(k) = R(R(k)) until every chain is collapsed
    int changed = 0;
    for (int32_t k = tid; k < n; k += kShufThreads) {
      const uint16_t a = r[k], b = r[a];
      if (b != a) {
        r[k] = b;
        changed = 1;
      }
    }
    if (!__syncthreads_or(changed)) break;
  }
  const int32_t first0 = n > 1 && cnt[0] > 0 ? (int32_t)srt[0] : -1;
  const int64_t q0 = M.part_base ? M.part_base[p] : 0;
  for (int32_t k = tid; k < n; k += kShufThreads) {
    const int32_t sc = k == 0 ? first0 : ord[k];
    const int32_t v = sc >= 0 ? (int32_t)r[sc] : (k == 0 ? 0 : ~sc);
    ord[k] = v;
    if (M.src) M.src[q0 + k] = base + v;
    if (M.slots) M.slots[q0 + k] = base + k;
    if (M.dstq) M.dstq[q0 + v] = q0 + k;
  }
}

// ---------------------------------------------------------------------------------------------
// layout + gather
// ---------------------------------------------------------------------------------------------
// src[q]: the planner slot of output pair q (partition shuffle applied); slots[q]: the q-th
// slot in planner order (every partition's slots base .. base + np - 1), so the per-slot passes
// read the slot-indexed arrays front to back instead of in shuffled order.
// (any output may be null)
// dstq[i]: the output position of the i-th pair in planner order (the inverse of src), for the
// mask replay that also writes each pair's gather record.
__global__ void map_pairs_kernel(const int64_t* kd_off, const int64_t* kp_off, int32_t dup,
                                 const int64_t* part_pair_base, const int32_t* order, int64_t* src,
                                 int64_t* slots, int64_t* dstq) {
  const int p = blockIdx.x;
  const int64_t base = (int64_t)dup * kd_off[kp_off[p]];
  const int64_t q0 = part_pair_base[p], n = part_pair_base[p + 1] - q0;
  for (int64_t k = threadIdx.x; k < n; k += blockDim.x) {
    if (src) src[q0 + k] = base + order[base + k];
    if (slots) slots[q0 + k] = base + k;
    if (dstq) dstq[q0 + order[base + k]] = q0 + k;
  }
}

// the largest partition's pair count (the partition shuffle's LDS size)
__global__ void max_pairs_kernel(const int64_t* np, int64_t n, unsigned long long* out) {
  int64_t m = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    m = np[i] > m ? np[i] : m;
  if (m) atomicMax(out, (unsigned long long)m);
}

struct Identity {
  const int64_t* v;
  __device__ int64_t operator()(int64_t i) const { return v[i]; }
};

// Per output pair, everything the gather needs, in output order: the A and B windows in the dense
// token array, the lengths and is_random_next, and the masks' place in the mask pool. Built one
// lane per pair (src -> descriptor -> sentence offsets: every load of a wave in flight at once),
// so the scans and the gather read it front to back instead of chasing src[q] themselves.
struct alignas(16) GatherRec {
  int64_t aoff, boff, moff;
  int32_t na, nb_rn, nm, pad;
};

__global__ void __launch_bounds__(256) pair_prep_kernel(const int64_t* __restrict__ src, int64_t n,
                                                        const PairDesc* __restrict__ desc,
                                                        const int64_t* __restrict__ kscan,
                                                        const int32_t* __restrict__ nmask,
                                                        const int64_t* __restrict__ moff,
                                                        GatherRec* __restrict__ rec,
                                                        int2* __restrict__ cnt) {
  // (XCD-contiguous blocks: a partition's pairs share one L2 for its descriptors and offsets)
  const int64_t q = xcd_block(blockIdx.x, gridDim.x) * 256 + threadIdx.x;
  if (q >= n) return;
  const int64_t slot = src[q];
  const PairDesc d = desc[slot];
  GatherRec r;
  r.aoff = kscan[d.a_ks] + d.a_front;
  r.boff = kscan[d.b_ks] + d.b_front;
  // masks: the native path's arrays (none: no masking; the replay path's records come from
  // fy_resolve_kernel)
  r.moff = nmask ? moff[slot] : 0;
  r.na = d.na;
  r.nb_rn = d.nb_rn;
  r.nm = nmask ? nmask[slot] : 0;
  r.pad = 0;
  rec[q] = r;
  cnt[q] = make_int2(r.na + (r.nb_rn & 0x7FFFFFFF), r.nm);  // compact input of the two scans
}

struct PairTokens {
  const int2* c;
  __device__ int64_t operator()(int64_t q) const { return c[q].x; }
};
struct PairCounts {  // both, for scan_exclusive2
  const int2* c;
  __device__ Sum2 operator()(int64_t q) const {
    const int2 v = c[q];
    return Sum2{v.x, v.y};
  }
};

// Kept tokens packed densely in kept-sentence order: kept sentence k's pieces are
// dense[kscan[k] .. kscan[k+1]). A pair's A (and B) window is then one contiguous run
// dense[kscan[a_ks] + a_front ..+ na), because a span only ever covers consecutive kept
// sentences of one document. One wave per 64 kept sentences; 64-token output chunks are stored
// coalesced, each lane finding its sentence among the few that overlap the chunk.
__global__ void __launch_bounds__(256) densify_kernel(const int64_t* __restrict__ ks_start,
                                                      const int32_t* __restrict__ ks_len,
                                                      const int64_t* __restrict__ kscan, int64_t n,
                                                      const int32_t* __restrict__ ids,
                                                      IdPtr dense) {
  const int64_t k0 = ((int64_t)blockIdx.x * 4 + wave_id()) * 64;
  if (k0 >= n) return;
  densify_group(k0, ks_start, ks_len, kscan, n, ids, dense);
}


struct GatherArgs {
  const void* dense;     // kept tokens, packed (IdT)
  const GatherRec* rec;  // per output pair (pair_prep_kernel)
  // masks: positions + replacements at rec.moff (any order; ranks are taken from the bitmap)
  const uint16_t* mpos;
  const int32_t* mtok;
  int32_t masking;
  int64_t n_pairs;
  const int64_t* tok_off;
  const int64_t* pos_off;
  void* out_tok;  // IdT
  int32_t* len_a;
  uint8_t* is_rn;
  uint16_t* out_pos;
  void* out_lab;  // IdT
  int64_t* out_tok_off;  // the caller's copies of tok_off / pos_off (may be null)
  int64_t* out_pos_off;
};

constexpr int kMaxSeqGather = 4096;
constexpr int kGWaves = 4;

// LDS of the gather per pair in flight: the decision table indexed by output token x (seqp =
// seq rounded up to 128 entries of int32, kNoMask where x is not masked) and the staging rows
// of one pass's masked positions and labels by rank (128 each, then one trash entry per lane).
constexpr int32_t kNoMask = INT32_MIN;
constexpr int kStageRows = 128;  // + 32 trash entries, one per lane of the half-wave
struct GatherLds {
  int32_t seqp;
  int32_t ib;  // bytes per label id (the staging row's width)
  int32_t db;  // bytes per decision-table entry: 4 (int32), 2 in gather16_kernel (16-bit ids)
  __host__ __device__ size_t per_pair() const {
    return (size_t)db * seqp + (size_t)(kStageRows + 32) * (size_t)(2 + ib);
  }
};
// gather16_kernel's 16-bit decision table: a token id, or one of two values no id takes (the
// context uses 2-byte ids only for vocabs of <= 65,534 entries)
constexpr uint16_t kNoMask16 = 0xFFFFu, kKeep16 = 0xFFFEu;

// Replay masks, off the planner's sequential chain: one LANE per pair replays the recorded swaps
// of random.shuffle(cand_indexes) (draws j_i, i = nc-1 .. 1) on a lane-private LDS column and
// writes the candidates that end in slots 0 .. num-1, as positions of [CLS] A [SEP] B [SEP], in
// slot order (= the order of the planner's decisions) over the mask pool. Steps i >= num only
// move x[i] to x[j_i] (slot i is never read again); steps i < num finalise slot i = x[j_i].
// Column layout x[k * 64 + lane] keeps the 64 lanes' accesses in distinct banks.
struct ResolveArgs {
  const int64_t* src;  // slots in planner order (each pair once; mpos is addressed by moff)
  int64_t n_pairs;
  const PairDesc* desc;
  const SlotPool* spool;
  const void* jpool;   // 1- or 2-byte draws (the kernel's D)
  uint16_t* mpos;
  const int64_t* kscan;
  IdPtr dense;
  int32_t cls_id, sep_id;
  // with masking on the replay path, the pair's gather record and scan counts are written here
  // too, at its output position dstq[i] (what pair_prep_kernel does for the other paths: the
  // descriptor and slot record are already in registers, and planner order reads them front to
  // back); null otherwise
  const int64_t* dstq;
  GatherRec* rec;
  int2* cnt;
  int32_t col_rows;  // entries per lane column in LDS (seq rounded up to 16)
};

// A lane's column of LDS entries; 16-bit: x[k * LW + lane]; 8-bit (seq <= 256): dword k/4 of
// lane l at (k/4) * LW + l, so every access of the wave hits distinct banks either way.
template <typename T, int LW>
struct LaneCol;
template <int LW>
struct LaneCol<uint16_t, LW> {
  uint16_t* base;
  int lane;
  __device__ uint32_t get(int k) const { return base[k * LW + lane]; }
  __device__ void set(int k, uint32_t v) { base[k * LW + lane] = (uint16_t)v; }
  __device__ void iota(int n) {
    for (int k = 0; k < n; ++k) set(k, (uint32_t)k);
  }
};
template <int LW>
struct LaneCol<uint8_t, LW> {
  uint8_t* base;
  int lane;
  __device__ int at(int k) const { return ((k >> 2) * (4 * LW)) | (lane << 2) | (k & 3); }
  __device__ uint32_t get(int k) const { return base[at(k)]; }
  __device__ void set(int k, uint32_t v) { base[at(k)] = (uint8_t)v; }
  __device__ void iota(int n) {
    uint32_t* w = reinterpret_cast<uint32_t*>(base);
    for (int k = 0; k < n; k += 4)
      w[(k >> 2) * LW + lane] = (uint32_t)k | (uint32_t)(k + 1) << 8 | (uint32_t)(k + 2) << 16 |
                                (uint32_t)(k + 3) << 24;
  }
};

// D: draw type (uint8_t for target_seq_length <= 256, else uint16_t); a uint4 holds 16 / sizeof(D)
// draws. NG > 0: all of a pair's draws (nc <= NG * 16 / sizeof(D)) are loaded up front, NG uint4
// in flight per lane.
// LW: pairs (lanes) per workgroup of one wave. Long pairs run with LW < 64: a lane's column is
// seq entries, so at seq 512 a full wave holds 64 KB of LDS and only two fit a CU; fewer lanes
// per wave put more waves (more independent step chains) on each SIMD.
template <typename T, typename D, int NG, int LW = 64, bool kBF = false, int kRA = 0, int kPf = 4>
__global__ void __launch_bounds__(64) fy_resolve_kernel(ResolveArgs R) {
  extern __shared__ __attribute__((aligned(16))) uint8_t s_xb[];
  constexpr int kPerVec = 16 / (int)sizeof(D);  // draws per uint4
  const int lane = threadIdx.x;
  LaneCol<T, LW> x{reinterpret_cast<T*>(s_xb), lane};
  // (XCD-contiguous blocks: a partition's pairs, their kept-sentence offsets and records meet
  // in one L2)
  const int64_t q = xcd_block(blockIdx.x, gridDim.x) * LW + lane;
  // 16-bit columns, branch-free steps: the workgroup writes the identity into every column at
  // once, 8 rows (one entry per lane and row) per 16-byte store per lane, before any lane leaves
  // (a lane's own per-entry iota was ~20 % of the kernel's LDS instructions and half its scalar
  // ones; C3 profiles/r05n_*). Rows past a lane's nc are only touched by its padding steps.
  constexpr bool kCoopIota = kBF && sizeof(T) == 2 && LW == 16;
  if constexpr (kCoopIota) {
    const int rows = (int)(R.col_rows);
    uint4* base = reinterpret_cast<uint4*>(s_xb);
    for (int k0 = 0; k0 < rows; k0 += 8) {
      const uint32_t k = (uint32_t)(k0 + (lane >> 1)), kk = k | k << 16;
      base[2 * k + (lane & 1)] = make_uint4(kk, kk, kk, kk);  // row k = 32 bytes = 2 uint4
    }
    // lanes wrote rows of other lanes' columns: order the fill before any lane reads its own
    // column (a one-wave workgroup: the barrier is a wait on the LDS stores)
    __syncthreads();
  }
  if (q >= R.n_pairs) return;
  const int64_t slot = R.src[q];
  const int64_t oq = R.dstq ? R.dstq[q] : 0;
  // the whole 16-byte record and the descriptor in one round trip (a member-wise read split the
  // record around the early exit below)
  const uint4 spv = *reinterpret_cast<const uint4*>(R.spool + slot);
  const PairDesc d = R.desc[slot];
  const SlotPool sp{spv.x, spv.y, (int32_t)spv.z, (int32_t)spv.w};
  const int32_t num = sp.nmask;
  const int32_t nc = num > 0 ? sp.ncand : 0;  // (no early exit: it split the loads above)
  const int64_t jb = (int64_t)sp.joff16 << 4, mb = (int64_t)sp.moff8 << 3;
  const int32_t na = d.na, nb = d.nb_rn & 0x7FFFFFFF;
  const bool fast = nc == na + nb;
  const int64_t ao = R.kscan[d.a_ks] + d.a_front, bo = R.kscan[d.b_ks] + d.b_front;
  const uint4* jp = reinterpret_cast<const uint4*>(static_cast<const D*>(R.jpool) + jb);
  uint4* mp = reinterpret_cast<uint4*>(R.mpos + mb);
  uint4 acc = make_uint4(0u, 0u, 0u, 0u);  // slots [8h, 8h+8) collected from the top down
  // steps [8h, 8h+8): swap, or (i < num) finalise slot i; w = the two (1-byte draws) or four
  // (2-byte draws) dwords holding their draws
  auto group = [&](int h, const uint32_t* w) {
#pragma unroll
    for (int u = 7; u >= 0; --u) {
      const int i = 8 * h + u;
      if (i >= nc) continue;
      const int j = sizeof(D) == 1 ? (int)((w[u >> 2] >> (8 * (u & 3))) & 0xFFu)
                                   : (int)((w[u >> 1] >> (16 * (u & 1))) & 0xFFFFu);
      const uint32_t xi = x.get(i);
      if (i >= num) {
        if (i >= 1) x.set(j, xi);
      } else {
        const int y = i >= 1 ? (int)x.get(j) : (int)xi;  // slot 0 keeps x[0]
        if (i >= 1) x.set(j, xi);
        const uint32_t pos = (uint32_t)(fast ? (y < na ? y + 1 : y + 2) : y);
        // 128-bit shift register, newest at slot offset 0 (slots arrive in descending order)
        acc = make_uint4((acc.x << 16) | pos, (acc.y << 16) | (acc.x >> 16),
                         (acc.z << 16) | (acc.y >> 16), (acc.w << 16) | (acc.z >> 16));
      }
    }
    if (8 * h < num) mp[h] = acc;  // slots [8h, 8h+8) complete (the top group zero-padded)
  };
  // kBF: the same steps without exec-mask branches. The planner pads a pair's draw region
  // ([nc, nc rounded up to 16) hold j_i = i) and step 0 takes j = 0 (entry 0 of the region is
  // never a draw), so every step of a loaded vector is x[j] = x[i] unguarded (a padding step
  // rewrites x[i] onto itself); a group in which no
  // lane of the wave finalises a slot is that move alone (read, wait, write: ~2 VALU per
  // step); otherwise each step also reads y = x[j] before the write (i = 0: j = 0, y = x[0])
  // and keeps its position by select. Round 4's guarded steps spent ~10 scalar exec-mask
  // instructions and three branches per step.
  const int32_t padd = fast ? 1 : 0, thr = fast ? na : INT32_MAX;  // pos = y + padd + (y >= thr)
  // draw u of a group (step 8h + u); step 0 has none: j_0 = 0
  auto draw = [&](int h, const uint32_t* w, int u) -> int {
    const int j = sizeof(D) == 1 ? (int)((w[u >> 2] >> (8 * (u & 3))) & 0xFFu)
                                 : (int)((w[u >> 1] >> (16 * (u & 1))) & 0xFFFFu);
    return u == 0 && h == 0 ? 0 : j;
  };
  auto group_bf = [&](int h, const uint32_t* w) {
    if (__any(8 * h < num)) {
      uint32_t pos[8];
#pragma unroll
      for (int u = 7; u >= 0; --u) {
        const int i = 8 * h + u;
        const int j = draw(h, w, u);
        const uint32_t xi = x.get(i);
        const int y = (int)x.get(j);
        x.set(j, xi);
        pos[u] = i < num ? (uint32_t)(y + padd + (y >= thr ? 1 : 0)) : 0u;
      }
      if (8 * h < num)
        mp[h] = make_uint4(pos[0] | pos[1] << 16, pos[2] | pos[3] << 16, pos[4] | pos[5] << 16,
                           pos[6] | pos[7] << 16);
    } else if (kRA == 0) {
#pragma unroll
      for (int u = 7; u >= 0; --u) x.set(draw(h, w, u), x.get(8 * h + u));
    } else {
      // kRA reads ahead: x[i - kRA] is read before step i's write (the group's top kRA entries
      // at its start), so step u's read misses the writes of steps u + 1 .. min(u + kRA, 7),
      // which are forwarded from registers (the most recent wins)
      int jr[8];  // j - 8h: compared with the step offset u
      uint32_t r[8], v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) jr[u] = draw(h, w, u) - 8 * h;
#pragma unroll
      for (int u = 7; u >= 8 - kRA; --u) r[u] = x.get(8 * h + u);
#pragma unroll
      for (int u = 7; u >= 0; --u) {
        if (u - kRA >= 0) r[u - kRA] = x.get(8 * h + u - kRA);
        uint32_t val = r[u];
#pragma unroll
        for (int t = kRA; t >= 1; --t)  // oldest first
          if (u + t <= 7) val = jr[u + t] == u ? v[u + t] : val;
        v[u] = val;
        x.set(jr[u] + 8 * h, val);
      }
    }
  };
  // one uint4 of draws = kPerVec / 8 groups of 8 steps, processed top down
  auto vec = [&](int g, const uint4& v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    if (kBF) {
      if (sizeof(D) == 1) group_bf(2 * g + 1, w + 2);
      group_bf(sizeof(D) == 1 ? 2 * g : g, w);
    } else if (sizeof(D) == 1) {
      if (16 * g + 8 < nc) group(2 * g + 1, w + 2);
      group(2 * g, w);
    } else {
      group(g, w);
    }
  };
  const int nvec = (nc + kPerVec - 1) / kPerVec;
  if (NG > 0) {
    uint4 jv[NG > 0 ? NG : 1];
#pragma unroll
    for (int g = 0; g < NG; ++g)
      if (g < nvec) jv[g] = jp[g];
    if (!kCoopIota) x.iota(nc);  // (after the draws' loads are issued)
#pragma unroll
    for (int g = NG - 1; g >= 0; --g)
      if (g < nvec) vec(g, jv[g]);
  } else if (nvec > 0) {  // (a pair without masks has no draws to read)
    // four vectors of draws in flight: one vector ahead left each vector's global load latency
    // exposed every 8 steps (C3, seq 512: 93 -> 77.7 ms; eight ahead 80.1 ms, profiles/r04zj_*,
    // r04zk_*)
    auto ld = [&](int g) { return jp[g < 0 ? 0 : g]; };
    const int top = nvec - 1;
    uint4 rv[kPf];
#pragma unroll
    for (int u = 0; u < kPf; ++u) rv[u] = ld(top - u);
    if (!kCoopIota) x.iota(nc);
    for (int g = top; g >= 0; g -= kPf) {
#pragma unroll
      for (int u = 0; u < kPf; ++u) {
        if (g >= u) vec(g - u, rv[u]);
        rv[u] = ld(g - u - kPf);
      }
    }
  }
  if (R.rec) {
    GatherRec r;
    r.aoff = ao;
    r.boff = bo;
    r.moff = mb;
    r.na = na;
    r.nb_rn = d.nb_rn;
    r.nm = num;
    r.pad = 0;
    R.rec[oq] = r;
    R.cnt[oq] = make_int2(na + nb, num);
  }
  if (!fast && num > 0) {  // literal [CLS]/[SEP] in the pair: candidate index -> position via the tokens
    int k = 0;
    for (int t = 0; t < na + nb; ++t) {
      const int32_t tok = t < na ? R.dense.ld(ao + t) : R.dense.ld(bo + (t - na));
      if (tok != R.cls_id && tok != R.sep_id) x.set(k++, (uint32_t)(t < na ? t + 1 : t + 2));
    }
    uint16_t* m16 = R.mpos + mb;
    for (int c = 0; c < num; ++c) m16[c] = (uint16_t)x.get(m16[c]);
  }
}

// Gather: each half-wave emits K output pairs, 4 consecutive tokens per lane (128 per pass), so
// a wave has 2K pairs in flight with all their parameters in vector registers. Per pair:
// A = dense[kscan[a_ks] + a_front ..+ na), B likewise; output token x < na + nb comes from A
// (x < na, position x + 1) or B (position x + 2); a lane's 4 tokens are one 8- or 16-byte load
// and one non-temporal store except where they straddle A/B or the end. The pair's masks (pool,
// any order) fill a per-pair LDS decision table indexed by x (one plain LDS store per mask);
// each lane reads its 4 entries with one 16-byte LDS load. A masked token's rank (its place in
// the position-sorted masked_lm_positions / labels) is the half-wave's exclusive scan of the
// lanes' masked counts (one DPP scan for all K pairs, counts packed 16 bits apart) plus the
// masked elements before it in the lane; (position, label) go to an LDS staging row by rank and
// leave as two coalesced stores per pass (round 3 issued eight lane-masked 2-byte stores per
// pass from four ballots per element: that mask path was half the kernel, profiles/r04t_*).
// The caller's tok_off / pos_off are written here too (no device-to-device copies).
// 4 consecutive token ids (one lane's share of a pass): 16 bytes of int32 ids, 8 of uint16 ids
template <typename IdT>
struct Tok4;
template <>
struct Tok4<int32_t> {
  typedef int32_t type __attribute__((ext_vector_type(4), aligned(4)));
};
template <>
struct Tok4<uint16_t> {
  typedef uint16_t type __attribute__((ext_vector_type(4), aligned(2)));
};
// The raw load of 4 ids, and the blend "element e from A iff e < ra" (ra = A elements left)
__device__ inline uint2 blend4(uint2 a, uint2 b, int32_t ra) {
  const int32_t bits = ra <= 0 ? 0 : ra >= 4 ? 64 : 16 * ra;
  const uint32_t mlo = bits >= 32 ? ~0u : (1u << bits) - 1u;
  const uint32_t mhi = bits >= 64 ? ~0u : bits <= 32 ? 0u : (1u << (bits - 32)) - 1u;
  return make_uint2((a.x & mlo) | (b.x & ~mlo), (a.y & mhi) | (b.y & ~mhi));
}
__device__ inline int4 blend4(int4 a, int4 b, int32_t ra) {
  return make_int4(0 < ra ? a.x : b.x, 1 < ra ? a.y : b.y, 2 < ra ? a.z : b.z, 3 < ra ? a.w : b.w);
}
template <typename IdT>
using Raw4 = std::conditional_t<sizeof(IdT) == 2, uint2, int4>;

template <int K, typename IdT>
__global__ void __launch_bounds__(64 * kGWaves, 1) gather_kernel(GatherArgs G, GatherLds Lg) {
  static_assert(K == 1 || K == 2, "masked counts of K pairs are packed 16 bits apart");
  using tok4_t = typename Tok4<IdT>::type;
  const IdT* __restrict__ dense = static_cast<const IdT*>(G.dense);
  extern __shared__ __attribute__((aligned(16))) uint8_t g_smem[];
  const int w = wave_id(), lane = threadIdx.x & 63, h = lane >> 5, sl = lane & 31;
  // XCD-contiguous blocks: the pairs of one partition (which read its dense tokens dup times over)
  // and their mask pool lines meet in one L2
  const int64_t wg = xcd_block((int64_t)blockIdx.y * gridDim.x + blockIdx.x, (int64_t)gridDim.x * gridDim.y);
  const int64_t q0 = (wg * kGWaves + w) * 2 * K;  // pairs q0 + 2k + h

  int64_t tof[K], aoff[K], boff[K], po[K], mb[K];
  int32_t na[K], nb[K], rk[K], nm[K];
  int32_t* dec[K];
  uint16_t* spos[K];
  IdT* slab[K];
  GatherRec rc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {  // every pair's loads in flight before any is used
    const int64_t q = q0 + 2 * k + h;
    const bool act = q < G.n_pairs;
    rc[k] = act ? G.rec[q] : GatherRec{0, 0, 0, 0, 0, 0, 0};
    tof[k] = act ? G.tok_off[q] : 0;
    po[k] = (G.masking && act) ? G.pos_off[q] : 0;
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int64_t q = q0 + 2 * k + h;
    const GatherRec& r = rc[k];
    na[k] = r.na;
    nb[k] = r.nb_rn & 0x7FFFFFFF;
    aoff[k] = r.aoff;
    boff[k] = r.boff;
    mb[k] = r.moff;
    nm[k] = G.masking ? r.nm : 0;
    rk[k] = 0;
    uint8_t* pb = g_smem + (((size_t)w * K + k) * 2 + h) * Lg.per_pair();
    dec[k] = reinterpret_cast<int32_t*>(pb);
    spos[k] = reinterpret_cast<uint16_t*>(pb + 4 * (size_t)Lg.seqp);
    slab[k] = reinterpret_cast<IdT*>(pb + 4 * (size_t)Lg.seqp + 2 * (kStageRows + 32));
    if (sl == 0 && q < G.n_pairs) {
      G.len_a[q] = na[k];
      G.is_rn[q] = (uint8_t)((uint32_t)r.nb_rn >> 31);
      if (G.out_tok_off) {
        G.out_tok_off[q] = tof[k];
        if (q + 1 == G.n_pairs) G.out_tok_off[q + 1] = tof[k] + na[k] + nb[k];
      }
      if (G.out_pos_off && G.masking) {
        G.out_pos_off[q] = po[k];
        if (q + 1 == G.n_pairs) G.out_pos_off[q + 1] = po[k] + nm[k];
      }
    }
  }
  // a lane's 4 tokens: one load from A and one from B, each at the offset of token x in that
  // window (dense is padded by 4 tokens on both sides, so a load overhanging its window stays in
  // bounds); element e comes from A iff x + e < na. Both loads are issued unconditionally (an
  // unneeded one reads the window start) and blended only when the pass needs the tokens: a
  // conditional load made the compiler wait for it inside its branch, before the next pair's
  // loads were issued.
  using raw_t = Raw4<IdT>;
  raw_t ta[K], tb[K];
  auto issue_tokens = [&](int32_t x) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int32_t n = na[k] + nb[k], bx = x - na[k];
      ta[k] = *reinterpret_cast<const raw_t*>(dense + aoff[k] + (x < na[k] ? x : 0));
      tb[k] = *reinterpret_cast<const raw_t*>(dense + boff[k] + (bx >= -3 && x < n ? bx : 0));
    }
  };
  auto finish_tokens = [&](int32_t x, tok4_t* v) {
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = __builtin_bit_cast(tok4_t, blend4(ta[k], tb[k], na[k] - x));
  };
  tok4_t v[K];
  issue_tokens(4 * sl);  // the first pass's tokens are in flight while the tables fill
  if (G.masking) {
#pragma unroll
    for (int k = 0; k < K; ++k)
      for (int i = 4 * sl; i < Lg.seqp; i += 128)
        *reinterpret_cast<int4*>(dec[k] + i) = make_int4(kNoMask, kNoMask, kNoMask, kNoMask);
    wave_sync();
#pragma unroll
    for (int k = 0; k < K; ++k)
      for (int j = sl; j < nm[k]; j += 32) {
        const int p = G.mpos[mb[k] + j];  // position in [CLS] A [SEP] B [SEP]: never a literal
        dec[k][p <= na[k] ? p - 1 : p - 2] = G.mtok[mb[k] + j];
      }
    wave_sync();
  }
  for (int32_t cb = 0;; cb += 128) {
    const int32_t x = cb + 4 * sl;
    if (cb > 0) issue_tokens(x);
    finish_tokens(x, v);
    bool more = false;
    if (G.masking) {
      int4 d4[K];
      uint32_t m4[K], packed = 0;
#pragma unroll
      for (int k = 0; k < K; ++k) {  // (x < seqp: every pass starts below the longest pair)
        d4[k] = *reinterpret_cast<const int4*>(dec[k] + x);
        m4[k] = (d4[k].x != kNoMask ? 1u : 0u) | (d4[k].y != kNoMask ? 2u : 0u) |
                (d4[k].z != kNoMask ? 4u : 0u) | (d4[k].w != kNoMask ? 8u : 0u);
        packed |= (uint32_t)__popc(m4[k]) << (16 * k);
      }
      // per half-wave exclusive scan of the packed counts (<= 128 per pair and pass)
      const uint32_t inc = wave_incl_scan(packed);
      const uint32_t lo_tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, 31);
      const uint32_t all_tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
      const uint32_t excl = inc - packed - (h ? lo_tot : 0u);
      const uint32_t tots = h ? all_tot - lo_tot : lo_tot;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        int32_t r = (int32_t)((excl >> (16 * k)) & 0xFFFFu);
        const int32_t dd[4] = {d4[k].x, d4[k].y, d4[k].z, d4[k].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {  // branch-free: an unmasked element writes the lane's trash entry
          const bool mk = (m4[k] >> e) & 1u;
          const int32_t xe = x + e, at = mk ? r : kStageRows + sl;
          spos[k][at] = (uint16_t)(xe < na[k] ? xe + 1 : xe + 2);
          slab[k][at] = v[k][e];
          v[k][e] = mk && dd[e] != kKeep ? (IdT)dd[e] : v[k][e];
          r += mk ? 1 : 0;
        }
      }
      wave_sync();
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int32_t tot = (int32_t)((tots >> (16 * k)) & 0xFFFFu);
        for (int32_t i = sl; i < tot; i += 32) {
          G.out_pos[po[k] + rk[k] + i] = spos[k][i];
          static_cast<IdT*>(G.out_lab)[po[k] + rk[k] + i] = slab[k][i];
        }
        rk[k] += tot;
      }
      wave_sync();  // (the staging rows are rewritten by the next pass)
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int32_t n = na[k] + nb[k];
      // non-temporal: the output is streamed, never re-read by this step
      IdT* out = static_cast<IdT*>(G.out_tok) + tof[k];
      if (x + 3 < n) {
        __builtin_nontemporal_store(v[k], reinterpret_cast<tok4_t*>(out + x));
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (x + e < n) __builtin_nontemporal_store(v[k][e], out + x + e);
      }
      more |= n > cb + 128;
    }
    if (!ballot(more)) break;
  }
}

typedef uint16_t Tok8 __attribute__((ext_vector_type(8), aligned(2)));
__device__ inline uint4 blend8(uint4 a, uint4 b, int32_t ra) {  // element e from A iff e < ra
  const int32_t bits = ra <= 0 ? 0 : ra >= 8 ? 128 : 16 * ra;
  auto m = [&](int d) -> uint32_t {
    const int32_t t = bits - 32 * d;
    return t >= 32 ? ~0u : t <= 0 ? 0u : (1u << t) - 1u;
  };
  const uint32_t m0 = m(0), m1 = m(1), m2 = m(2), m3 = m(3);
  return make_uint4((a.x & m0) | (b.x & ~m0), (a.y & m1) | (b.y & ~m1), (a.z & m2) | (b.z & ~m2),
                    (a.w & m3) | (b.w & ~m3));
}

// The gather for 16-bit ids: LP = 16 or 8 lanes per output pair (4 or 8 pairs per wave), 128 / LP
// consecutive tokens per lane (16-byte loads from A and B, 16-byte non-temporal stores). Against
// gather_kernel<2, uint16_t> (a half-wave per pair, 4 tokens per lane, two pairs per lane) a pair
// costs fewer lanes and a lane holds one pair's registers, so more pairs are in flight per SIMD
// while the per-wave load chain (record -> tokens and masks -> stores) stays the same: 33.3 ->
// 29.5 ms per 10 GB step at LP = 16 (profiles/r04zd_*); LP = 8 needs 95 VGPRs and 37 KB of LDS
// per 4-wave block, runs at 4 waves/SIMD and took 35.3 ms (r04ze). The mask path is the same
// decision table by output token (16-byte LDS reads), ranks from an LP-lane DPP scan of the
// lanes' masked counts, and staged coalesced stores.
template <int LP>
struct G16 {
  static constexpr int kNT = 128 / LP;  // tokens per lane per pass
  static constexpr int kNV = kNT / 8;   // 16-byte vectors per lane
};

// inclusive scan of v over LP-lane segments (LP = 8 or 16) and the segment's total
template <int LP>
__device__ inline uint32_t seg_scan(uint32_t v, int lane, uint32_t* tot) {
  uint32_t inc = v;  // 16-lane row scan (row_shr 1, 2, 4, 8)
  inc = scan_step<0x111, 0xF, true>(inc);
  inc = scan_step<0x112, 0xF, true>(inc);
  inc = scan_step<0x114, 0xF, true>(inc);
  inc = scan_step<0x118, 0xF, true>(inc);
  const uint32_t r15 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x15F, 0xF, 0xF, false);  // row_share:15
  if (LP == 16) {
    *tot = r15;
    return inc;
  }
  const uint32_t r7 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x157, 0xF, 0xF, false);  // row_share:7
  const bool hi = (lane & 8) != 0;
  *tot = hi ? r15 - r7 : r7;
  return hi ? inc - r7 : inc;
}

template <int LP>
__global__ void __launch_bounds__(64 * kGWaves, 1) gather16_kernel(GatherArgs G, GatherLds Lg) {
  constexpr int NT = G16<LP>::kNT, NV = G16<LP>::kNV, PW = 64 / LP;  // PW pairs per wave
  const uint16_t* __restrict__ dense = static_cast<const uint16_t*>(G.dense);
  uint16_t* __restrict__ out_tok = static_cast<uint16_t*>(G.out_tok);
  uint16_t* __restrict__ out_lab = static_cast<uint16_t*>(G.out_lab);
  extern __shared__ __attribute__((aligned(16))) uint8_t g_smem[];
  const int w = wave_id(), lane = threadIdx.x & 63, qw = lane / LP, ql = lane % LP;
  // XCD-contiguous blocks (see gather_kernel)
  const int64_t wg = xcd_block((int64_t)blockIdx.y * gridDim.x + blockIdx.x, (int64_t)gridDim.x * gridDim.y);
  const int64_t q = (wg * kGWaves + w) * PW + qw;
  const bool act = q < G.n_pairs;
  const GatherRec r = act ? G.rec[q] : GatherRec{0, 0, 0, 0, 0, 0, 0};
  const int64_t tof = act ? G.tok_off[q] : 0;
  const int64_t po = (G.masking && act) ? G.pos_off[q] : 0;
  const int32_t na = r.na, nb = r.nb_rn & 0x7FFFFFFF, n = na + nb;
  const int32_t nm = G.masking ? r.nm : 0;
  const int64_t mb = r.moff;
  uint8_t* pb = g_smem + ((size_t)w * PW + qw) * Lg.per_pair();
  uint16_t* dec = reinterpret_cast<uint16_t*>(pb);
  uint16_t* spos = reinterpret_cast<uint16_t*>(pb + 2 * (size_t)Lg.seqp);
  uint16_t* slab = reinterpret_cast<uint16_t*>(pb + 2 * (size_t)Lg.seqp + 2 * (kStageRows + 32));
  if (ql == 0 && act) {
    G.len_a[q] = na;
    G.is_rn[q] = (uint8_t)((uint32_t)r.nb_rn >> 31);
    if (G.out_tok_off) {
      G.out_tok_off[q] = tof;
      if (q + 1 == G.n_pairs) G.out_tok_off[q + 1] = tof + n;
    }
    if (G.out_pos_off && G.masking) {
      G.out_pos_off[q] = po;
      if (q + 1 == G.n_pairs) G.out_pos_off[q + 1] = po + nm;
    }
  }
  // both NT-token loads unconditional (an unneeded one reads the window start; dense is padded
  // by 8 tokens on both sides and a B load starts at most 7 tokens before its window, an A load
  // overhangs only by the tokens a shorter A leaves, which the next 8-token vector's select
  // drops), blended when the pass needs them
  uint4 ta[NV], tb[NV];
  auto issue = [&](int32_t x) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int32_t xk = x + 8 * k, bx = xk - na;
      ta[k] = *reinterpret_cast<const uint4*>(dense + r.aoff + (xk < na ? xk : 0));
      tb[k] = *reinterpret_cast<const uint4*>(dense + r.boff + (bx >= -7 && xk < n ? bx : 0));
    }
  };
  issue(NT * ql);
  int32_t rk = 0;
  if (G.masking) {
    for (int i = 8 * ql; i < Lg.seqp; i += 8 * LP)
      *reinterpret_cast<uint4*>(dec + i) = make_uint4(~0u, ~0u, ~0u, ~0u);  // kNoMask16
    wave_sync();
    for (int j = ql; j < nm; j += LP) {
      const int p = G.mpos[mb + j];  // position in [CLS] A [SEP] B [SEP]: never a literal
      const int32_t t = G.mtok[mb + j];
      dec[p <= na ? p - 1 : p - 2] = t == kKeep ? kKeep16 : (uint16_t)t;
    }
    wave_sync();
  }
  for (int32_t cb = 0;; cb += 128) {
    const int32_t x = cb + NT * ql;
    if (cb > 0) issue(x);
    Tok8 v[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = __builtin_bit_cast(Tok8, blend8(ta[k], tb[k], na - x - 8 * k));
    if (G.masking) {
      uint32_t dd[NT];
#pragma unroll
      for (int k = 0; k < NT / 8; ++k) {  // (x < seqp, as in gather_kernel)
        const uint4 d = *reinterpret_cast<const uint4*>(dec + x + 8 * k);
        const uint32_t dw[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) dd[8 * k + e] = (dw[e >> 1] >> (16 * (e & 1))) & 0xFFFFu;
      }
      uint32_t mk = 0;
#pragma unroll
      for (int e = 0; e < NT; ++e) mk |= dd[e] != kNoMask16 ? 1u << e : 0u;
      const uint32_t c = (uint32_t)__popc(mk);
      uint32_t tot;
      const uint32_t inc = seg_scan<LP>(c, lane, &tot);
      int32_t rr = (int32_t)(inc - c);
#pragma unroll
      for (int e = 0; e < NT; ++e) {
        // only masked elements write their staging entries (exec-masked stores). Writing every
        // element, the unmasked ones to a per-lane trash entry, was 70 % of the kernel's LDS bank
        // conflicts (two lanes per dword, four pairs per wave on the same banks) at the same time
        // per launch (profiles/r06w_gather_lds_attribution.txt)
        const bool m = (mk >> e) & 1u;
        const int32_t xe = x + e;
        if (m) {
          spos[rr] = (uint16_t)(xe < na ? xe + 1 : xe + 2);
          slab[rr] = v[e >> 3][e & 7];
        }
        v[e >> 3][e & 7] = m && dd[e] != kKeep16 ? (uint16_t)dd[e] : v[e >> 3][e & 7];
        rr += m ? 1 : 0;
      }
      wave_sync();
      for (int32_t i = ql; i < (int32_t)tot; i += LP) {
        G.out_pos[po + rk + i] = spos[i];
        out_lab[po + rk + i] = slab[i];
      }
      rk += (int32_t)tot;
      wave_sync();  // (the staging rows are rewritten by the next pass)
    }
    uint16_t* out = out_tok + tof;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int32_t xk = x + 8 * k;
      if (xk + 7 < n) {
        __builtin_nontemporal_store(v[k], reinterpret_cast<Tok8*>(out + xk));
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (xk + e < n) __builtin_nontemporal_store(v[k][e], out + xk + e);
      }
    }
    if (!ballot(n > cb + 128)) break;
  }
}

}  // namespace
}  // namespace lddl

using namespace lddl;

// Device-resident plan of one batch of partitions (library-owned temporaries).
struct lddl_pairs {
  int device = 0;
  int32_t masking = 0, max_pred = 0, seq = 0, cls_id = -1, sep_id = -1;
  int64_t n_part = 0, n_pairs = 0, n_tokens = 0, n_masked = 0, n_kept_sent = 0, n_kept_doc = 0;
  DevArena* arena = nullptr;  // the context's block cache (the context outlives its plans)
  std::vector<DevArena::Block> allocs;
  // views
  int64_t *ks_start = nullptr, *kd_off = nullptr, *kp_off = nullptr, *kscan = nullptr;
  int32_t* ks_len = nullptr;
  IdPtr dense{nullptr, 4};  // kept tokens, packed in kept-sentence order (id_bytes each)
  PairDesc* desc = nullptr;
  int32_t *order = nullptr, *nmask = nullptr, *mtok = nullptr;
  uint16_t* mpos = nullptr;
  int64_t* moff = nullptr;
  int64_t *src = nullptr, *tok_off = nullptr, *pos_off = nullptr;
  GatherRec* rec = nullptr;  // per output pair (pair_prep_kernel)
  int64_t* part_base = nullptr;  // [n_part + 1] first output pair of each partition
  hipEvent_t ev[2] = {nullptr, nullptr};  // around the last plan_replay_kernel launch

  template <typename T>
  int alloc(T** p, int64_t n, hipStream_t st) {
    DevArena::Block b;
    LDDL_HIP(arena->take(sizeof(T) * (size_t)(n > 0 ? n : 1), st, b));
    *p = static_cast<T*>(b.p);
    allocs.push_back(b);
    return 0;
  }
  void free_one(void* p, hipStream_t st) {  // return one block early (re-plan)
    for (size_t i = 0; i < allocs.size(); ++i)
      if (allocs[i].p == p) {
        arena->give(allocs[i], st);
        allocs.erase(allocs.begin() + (ptrdiff_t)i);
        return;
      }
  }
  void release(hipStream_t st) {
    for (DevArena::Block& b : allocs) arena->give(b, st);
    allocs.clear();
    for (hipEvent_t& e : ev)
      if (e) {
        (void)hipEventDestroy(e);
        e = nullptr;
      }
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

// ceil(p * 2^53): random() < p  <=>  N < this (N = 53-bit integer behind random())
static uint64_t short_threshold(double p) {
  if (!(p > 0)) return 0;
  if (p >= 1) return 1ull << 53;
  return (uint64_t)ceil(ldexp(p, 53));
}

struct I32 {
  const int32_t* v;
  __device__ int64_t operator()(int64_t i) const { return v[i]; }
};

// LDDL_RNG_NATIVE control plane: count pass, unit scan, emit pass, mask offsets + masks, order.
static int plan_native(lddl_pairs* P, lddl_ctx* c, const lddl_pair_params* prm,
                       const int64_t* d_part_seed, int64_t n_part, hipStream_t st) {
  NativeArgs A{};
  A.ks_len = P->ks_len;
  A.kd_off = P->kd_off;
  A.kp_off = P->kp_off;
  A.kscan = P->kscan;
  A.dense = P->dense;
  A.part_seed = d_part_seed;
  A.n_part = n_part;
  int64_t kp_ends[2] = {0, 0};  // kept documents covered by the partitions
  unsigned long long need_max = 0, *d_need;
  int rc;
  if ((rc = P->alloc(&d_need, 1, st))) return rc;
  LDDL_HIP(hipMemsetAsync(d_need, 0, 8, st));
  if (n_part)
    hipLaunchKernelGGL(native_part_need_kernel, dim3((unsigned)((n_part + 255) / 256)), dim3(256), 0, st,
                       P->kp_off, P->kd_off, n_part, d_need);
  LDDL_HIP(hipMemcpyAsync(&kp_ends[0], P->kp_off, 8, hipMemcpyDeviceToHost, st));
  LDDL_HIP(hipMemcpyAsync(&kp_ends[1], P->kp_off + n_part, 8, hipMemcpyDeviceToHost, st));
  LDDL_HIP(hipMemcpyAsync(&need_max, d_need, 8, hipMemcpyDeviceToHost, st));
  LDDL_HIP(hipStreamSynchronize(st));
  A.unit0 = (int64_t)prm->dup * kp_ends[0];
  A.n_units = (int64_t)prm->dup * (kp_ends[1] - kp_ends[0]);
  A.native_seed = prm->native_seed;
  A.k_short = short_threshold(prm->short_seq_prob);
  A.seq = prm->seq;
  A.dup = prm->dup;
  A.masking = prm->masking;
  A.cls_id = c->tab.special_id[kCls];
  A.sep_id = c->tab.special_id[kSep];
  A.mask_id = c->tab.special_id[kMask];
  A.vocab_size = c->vocab_size;
  A.ratio = prm->masked_lm_ratio;
  const int64_t nu = A.n_units;
  // walk tables in LDS up to 96 KB per workgroup; larger partitions read a global prefix
  int64_t kLdsWordsCap = 24576;
  if (const char* e = getenv("LDDL_NATIVE_LDS_WORDS")) kLdsWordsCap = atoll(e);  // tests: global path
  const int32_t lds_words = (int32_t)std::max<int64_t>(
      1, std::min<int64_t>((int64_t)need_max, kLdsWordsCap));
  int64_t *uoff, *scr, *g_pre = nullptr;
  if ((rc = P->alloc(&A.ucnt, nu, st)) || (rc = P->alloc(&uoff, nu + 1, st)) ||
      (rc = P->alloc(&scr, scan_scratch_elems(std::max(nu, P->n_kept_sent) + 1), st)))
    return rc;
  if ((int64_t)need_max > kLdsWordsCap) {
    if ((rc = P->alloc(&g_pre, P->n_kept_sent + 1, st))) return rc;
    LDDL_HIP(scan_exclusive(KeptLenOnly{P->ks_len}, P->n_kept_sent, g_pre, scr, st));
  }
  LDDL_HIP(hipEventRecord(P->ev[0], st));
  const size_t lds_bytes = (size_t)4 * lds_words;
  if (n_part && nu)
    hipLaunchKernelGGL(plan_native_kernel<false>, dim3((unsigned)n_part), dim3(kNativeThreads), lds_bytes,
                       st, A, g_pre, lds_words);
  LDDL_HIP(hipGetLastError());
  LDDL_HIP(scan_exclusive(Identity{A.ucnt}, nu, uoff, scr, st));
  LDDL_HIP(hipMemcpyAsync(&P->n_pairs, uoff + nu, 8, hipMemcpyDeviceToHost, st));
  LDDL_HIP(hipStreamSynchronize(st));
  const int64_t n = P->n_pairs;
  A.uoff = uoff;
  A.n_pairs = n;
  if ((rc = P->alloc(&P->part_base, n_part + 1, st)) || (rc = P->alloc(&P->desc, n, st)) ||
      (rc = P->alloc(&A.ppart, n, st)) || (rc = P->alloc(&P->src, n, st)))
    return rc;
  if (prm->masking &&
      ((rc = P->alloc(&P->nmask, n, st)) || (rc = P->alloc(&A.ncand, n, st)) ||
       (rc = P->alloc(&P->moff, n + 1, st)) || (rc = P->alloc(&scr, scan_scratch_elems(n + 1), st))))
    return rc;
  hipLaunchKernelGGL(native_part_base_kernel, dim3((unsigned)((n_part + 256) / 256)), dim3(256), 0,
                     st, P->kp_off, n_part, prm->dup, uoff, P->part_base);
  A.part_base = P->part_base;
  A.desc = P->desc;
  A.nmask = P->nmask;
  if (n_part && nu)
    hipLaunchKernelGGL(plan_native_kernel<true>, dim3((unsigned)n_part), dim3(kNativeThreads), lds_bytes,
                       st, A, g_pre, lds_words);
  LDDL_HIP(hipGetLastError());
  const unsigned gp = (unsigned)((n + 255) / 256);
  if (prm->masking) {
    LDDL_HIP(scan_exclusive(I32{P->nmask}, n, P->moff, scr, st));
    LDDL_HIP(hipMemcpyAsync(&P->n_masked, P->moff + n, 8, hipMemcpyDeviceToHost, st));
    LDDL_HIP(hipStreamSynchronize(st));
    if ((rc = P->alloc(&P->mpos, P->n_masked, st)) || (rc = P->alloc(&P->mtok, P->n_masked, st)))
      return rc;
    A.moff = P->moff;
    A.mpos = P->mpos;
    A.mtok = P->mtok;
    A.words = (prm->seq + 31) / 32;
    // per wave: the 64 lanes' bitmaps + the staged masks of its 64 pairs (<= max_pred each);
    // up to 4 waves per workgroup within 64 KB of LDS
    const int32_t stage_cap = 64 * std::max(P->max_pred, 1);
    const size_t per_wave = (size_t)A.words * 64 * 4 + (size_t)stage_cap * 6;
    const int nwv = (int)std::max<size_t>(1, std::min<size_t>(4, 65536 / per_wave));
    if (n)
      hipLaunchKernelGGL(mask_native_kernel, dim3((unsigned)((n + 64 * nwv - 1) / (64 * nwv))),
                         dim3(64 * nwv), per_wave * nwv, st, A, stage_cap);
    LDDL_HIP(hipGetLastError());
  }
  A.src = P->src;
  if (n) hipLaunchKernelGGL(order_native_kernel, dim3(gp), dim3(256), 0, st, A);
  LDDL_HIP(hipGetLastError());
  LDDL_HIP(hipEventRecord(P->ev[1], st));
  return 0;
}

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
  if (prm->rng != LDDL_RNG_REPLAY && prm->rng != LDDL_RNG_NATIVE)
    LDDL_FAIL(-1, "unknown rng mode %d", prm->rng);
  const int32_t cls = c->tab.special_id[kCls], sep = c->tab.special_id[kSep],
                msk = c->tab.special_id[kMask];
  if (prm->masking && prm->seq > kMaxSeqGather)
    LDDL_FAIL(-1, "static masking supports target_seq_length <= %d", kMaxSeqGather);
  if (prm->masking && (cls < 0 || sep < 0 || msk < 0))
    LDDL_FAIL(-1, "static masking needs [CLS] [SEP] [MASK] in the vocab");
  hipStream_t st = as_stream(stream);
  auto* P = new lddl_pairs();
  P->device = c->device;
  P->arena = &c->arena;
  P->n_part = n_part;
  P->masking = prm->masking;
  P->seq = prm->seq;
  P->cls_id = cls;
  P->sep_id = sep;
  TRY(hipEventCreate(&P->ev[0]) == hipSuccess && hipEventCreate(&P->ev[1]) == hipSuccess
          ? 0 : (set_error("hipEventCreate failed"), -100));
  int64_t *ks_pos, *tok_pos, *kd_pos, *scratch, *part_npairs, *part_base;
  const int64_t nscr = 2 * scan_scratch_elems(std::max(n_sent, n_doc) + n_part + 1);  // (dual scans)
  TRY(P->alloc(&scratch, nscr, st));
  // compaction: kept-sentence index and token offset of every sentence in one scan
  TRY(P->alloc(&ks_pos, n_sent + 1, st));
  TRY(P->alloc(&tok_pos, n_sent + 1, st));
  if (scan_exclusive2(SentCounts{d_sent_len}, n_sent, ks_pos, tok_pos, scratch, st) != hipSuccess)
    TRY(-100);
  TRY(P->alloc(&kd_pos, n_doc + 1, st));
  if (scan_exclusive(KeepDoc{ks_pos, d_doc_sent_off}, n_doc, kd_pos, scratch, st) != hipSuccess)
    TRY(-100);
  int64_t h_counts[3];
  LDDL_HIP(hipMemcpyAsync(&h_counts[0], ks_pos + n_sent, 8, hipMemcpyDeviceToHost, st));
  LDDL_HIP(hipMemcpyAsync(&h_counts[1], kd_pos + n_doc, 8, hipMemcpyDeviceToHost, st));
  LDDL_HIP(hipMemcpyAsync(&h_counts[2], tok_pos + n_sent, 8, hipMemcpyDeviceToHost, st));
  LDDL_HIP(hipStreamSynchronize(st));
  P->n_kept_sent = h_counts[0];
  P->n_kept_doc = h_counts[1];
  const int64_t n_kept_tok = h_counts[2];  // (dropped sentences have no tokens)
  TRY(P->alloc(&P->ks_start, P->n_kept_sent, st));
  TRY(P->alloc(&P->ks_len, P->n_kept_sent, st));
  TRY(P->alloc(&P->kscan, P->n_kept_sent + 1, st));
  TRY(P->alloc(&P->kd_off, P->n_kept_doc + 1, st));
  TRY(P->alloc(&P->kp_off, n_part + 1, st));
  hipLaunchKernelGGL(scatter_sentences_kernel, dim3((unsigned)((n_sent + 256) / 256)), dim3(256), 0,
                     st, d_sent_off, d_sent_len, n_sent, ks_pos, tok_pos, P->ks_start, P->ks_len,
                     P->kscan);
  hipLaunchKernelGGL(scatter_docs_kernel, dim3((unsigned)((n_doc + 256) / 256)), dim3(256), 0, st,
                     d_doc_sent_off, n_doc, ks_pos, kd_pos, P->kd_off);
  unsigned long long* d_max_docs;
  TRY(P->alloc(&d_max_docs, 1, st));
  LDDL_HIP(hipMemsetAsync(d_max_docs, 0, 8, st));
  hipLaunchKernelGGL(part_offsets_kernel, dim3((unsigned)((n_part + 256) / 256)), dim3(256), 0, st,
                     d_part_doc_off, n_part, kd_pos, P->kp_off, d_max_docs);
  LDDL_HIP(hipGetLastError());
  // dense kept tokens
  unsigned long long max_docs = 0;
  LDDL_HIP(hipMemcpyAsync(&max_docs, d_max_docs, 8, hipMemcpyDeviceToHost, st));
  LDDL_HIP(hipStreamSynchronize(st));
  // 8 tokens of padding on both sides: the gather's 4- and 8-token loads may overhang a window
  {
    const int32_t ib = c->id_bytes();
    uint8_t* raw;
    TRY(P->alloc(&raw, (n_kept_tok + 16) * ib, st));
    P->dense = IdPtr{raw + 8 * ib, ib};
  }
  // replay mode: the planner launch's tail workgroups pack `dense` (plan_replay_kernel)
  const bool dense_in_plan = prm->rng == LDDL_RNG_REPLAY && n_part > 0;
  if (P->n_kept_sent && !dense_in_plan)
    hipLaunchKernelGGL(densify_kernel, dim3((unsigned)((P->n_kept_sent + 255) / 256)), dim3(256), 0,
                       st, P->ks_start, P->ks_len, P->kscan, P->n_kept_sent, d_ids, P->dense);
  LDDL_HIP(hipGetLastError());
  // plan
  const int64_t slots = (int64_t)prm->dup * P->n_kept_sent;
  int32_t max_pred = 0;
  if (prm->masking) {
    max_pred = (int32_t)rint((double)prm->seq * prm->masked_lm_ratio);
    if (max_pred < 1) max_pred = 1;
    if (max_pred > prm->seq) max_pred = prm->seq;

  }
  P->max_pred = max_pred;
  // the gather records + output-order scans (tok_off, pos_off) of the plan's pairs
  int2* pcnt = nullptr;
  int64_t* scr2 = nullptr;
  auto alloc_layout = [&](int64_t npairs) -> int {
    int rc;
    if ((rc = P->alloc(&P->tok_off, npairs + 1, st)) || (rc = P->alloc(&P->rec, npairs, st)) ||
        (rc = P->alloc(&pcnt, npairs, st)) || (rc = P->alloc(&scr2, 2 * scan_scratch_elems(npairs), st)))
      return rc;
    if (prm->masking && (rc = P->alloc(&P->pos_off, npairs + 1, st))) return rc;
    return 0;
  };
  auto scan_only = [&](hipStream_t s) -> int {  // tok_off (and pos_off) from the counts
    if (prm->masking)
      LDDL_HIP(scan_exclusive2(PairCounts{pcnt}, P->n_pairs, P->tok_off, P->pos_off, scr2, s));
    else
      LDDL_HIP(scan_exclusive(PairTokens{pcnt}, P->n_pairs, P->tok_off, scr2, s));
    return 0;
  };
  // gather records from the output order (src): the native path, and replay without masking
  auto prep_and_scan = [&](hipStream_t s) -> int {
    const int64_t npairs = P->n_pairs;
    if (npairs)
      hipLaunchKernelGGL(pair_prep_kernel, dim3((unsigned)((npairs + 255) / 256)), dim3(256), 0, s,
                         P->src, npairs, P->desc, P->kscan, prm->masking ? P->nmask : nullptr,
                         P->moff, P->rec, pcnt);
    LDDL_HIP(hipGetLastError());
    return scan_only(s);
  };
  if (prm->rng == LDDL_RNG_NATIVE) {
    TRY(plan_native(P, c, prm, d_part_seed, n_part, st));
  } else {
  int32_t* jseq;
  TRY(P->alloc(&P->desc, slots, st));
  TRY(P->alloc(&P->order, slots, st));
  TRY(P->alloc(&jseq, slots, st));
  TRY(P->alloc(&part_npairs, n_part + 1, st));
  SlotPool* spool = nullptr;
  if (prm->masking) TRY(P->alloc(&spool, slots, st));
  PlanArgs A{};
  A.kscan = P->kscan;
  A.ks_len = P->ks_len;
  A.kd_off = P->kd_off;
  A.kp_off = P->kp_off;
  A.ks_start = P->ks_start;
  A.ids = d_ids;
  A.dense = P->dense;
  A.n_kept_sent = dense_in_plan ? P->n_kept_sent : 0;
  A.n_part = (int32_t)n_part;
  A.n_dense_wg = 4096;
  A.part_seed = d_part_seed;
  A.seq = prm->seq;
  A.dup = prm->dup;
  A.masking = prm->masking;
  A.vocab_size = c->vocab_size;
  A.cls_id = cls;
  A.sep_id = sep;
  A.mask_id = msk;
  A.max_pred = max_pred;
  A.short_seq_prob = prm->short_seq_prob;
  A.ratio = prm->masked_lm_ratio;
  A.k_short = short_threshold(prm->short_seq_prob);
  A.seq_r64 = ((prm->seq + 63) / 64) * 64;
  A.desc = P->desc;
  A.jseq = jseq;
  A.spool = spool;
  A.part_npairs = part_npairs;
#ifdef LDDL_STAMPS
  uint64_t* d_stamps;
  TRY(P->alloc(&d_stamps, n_part * kStampRegions, st));
  LDDL_HIP(hipMemsetAsync(d_stamps, 0, 8 * n_part * kStampRegions, st));
  A.stamps = d_stamps;
  uint64_t* d_tl;
  TRY(P->alloc(&d_tl, n_part * 2, st));
  LDDL_HIP(hipMemsetAsync(d_tl, 0, 16 * n_part, st));
  A.tl = d_tl;
#endif
  if (prm->seq > 512) TRY((set_error("replay planner supports target_seq_length <= 512"), -1));
  const size_t lds = 4 * (kN + kLook) + 4 * (kDocLds + 4) + 16;  // ~4.8 KB: 7 waves/SIMD fit
  // pools: decisions (int32, shuffled order) and shuffle draws (uint16), sized from the kept
  // tokens (expected use ~0.15 * 1.5 and ~1.5 times dup * tokens); a plan that outgrows them
  // reports the exact sizes and is planned again (deterministic replay)
  unsigned long long* pool_ctl;  // [0] masks used, [1] overflow flag, [2] draws used, [3] max pairs
  TRY(P->alloc(&pool_ctl, 4, st));
  TRY(P->alloc(&part_base, n_part + 1, st));
  P->part_base = part_base;
  int64_t max_np = 1;
  int64_t cap = 0, jcap = 0;
  void* jpool = nullptr;
  const int jbytes = prm->seq <= 256 ? 1 : 2;  // every draw j_i < nc <= seq - 3
  if (prm->masking && n_sent) {
    const int64_t kept_tokens = n_kept_tok;
    cap = (int64_t)(2.0 * prm->masked_lm_ratio * prm->dup * (double)kept_tokens) +
          (int64_t)prm->dup * P->n_kept_sent / 2 + kPoolChunk * (n_part + 16);
    jcap = (int64_t)(1.6 * prm->dup * (double)kept_tokens) + 8 * slots +
           kPoolChunk * (n_part + 16);  // + the 16-entry alignment of every pair's draws
    if (const char* e = getenv("LDDL_AMD_MASK_POOL")) cap = atoll(e);  // tests: force a re-plan
  }
  // SlotPool keeps pool offsets as 32-bit multiples of 8 / 16 entries
  if (cap / 8 >= (int64_t)UINT32_MAX || jcap / 16 >= (int64_t)UINT32_MAX)
    TRY((set_error("batch too large for the mask pools (split it into smaller GPU batches)"), -1));
  for (int attempt = 0; n_part; ++attempt) {
    int32_t* mtok = nullptr;
    if (prm->masking) {
      LDDL_HIP(hipMemsetAsync(pool_ctl, 0, 32, st));
      TRY(P->alloc(&mtok, cap + 4, st));
      TRY(P->alloc(reinterpret_cast<uint8_t**>(&jpool), jbytes * (jcap + 16), st));
    }
    A.mtok = mtok;
    A.jpool = jpool;
    A.jbytes = jbytes;
    A.pool_cap = cap;
    A.jpool_cap = jcap;
    A.pool_used = pool_ctl;
    A.overflow = reinterpret_cast<int32_t*>(pool_ctl + 1);
    LDDL_HIP(hipEventRecord(P->ev[0], st));
    {
      const dim3 grid((unsigned)n_part + (A.n_kept_sent ? (unsigned)A.n_dense_wg : 0u));
      const bool docs_lds = max_docs + 1 <= (unsigned long long)kDocLds;
      if (docs_lds && jbytes == 1)
        hipLaunchKernelGGL((plan_replay_kernel<true, 1>), grid, dim3(64), lds, st, A);
      else if (docs_lds)
        hipLaunchKernelGGL((plan_replay_kernel<true, 2>), grid, dim3(64), lds, st, A);
      else if (jbytes == 1)
        hipLaunchKernelGGL((plan_replay_kernel<false, 1>), grid, dim3(64), lds, st, A);
      else
        hipLaunchKernelGGL((plan_replay_kernel<false, 2>), grid, dim3(64), lds, st, A);
    }
    LDDL_HIP(hipGetLastError());
    LDDL_HIP(hipEventRecord(P->ev[1], st));
    // pairs per partition -> output offsets and the largest count, read back with the pool
    // counters in the planner's one sync
    if (!prm->masking) LDDL_HIP(hipMemsetAsync(pool_ctl, 0, 32, st));
    if (scan_exclusive(Identity{part_npairs}, n_part, part_base, scratch, st) != hipSuccess) TRY(-100);
    hipLaunchKernelGGL(max_pairs_kernel, dim3(64), dim3(256), 0, st, part_npairs, n_part, pool_ctl + 3);
    unsigned long long ctl[4];
    LDDL_HIP(hipMemcpyAsync(ctl, pool_ctl, 32, hipMemcpyDeviceToHost, st));
    LDDL_HIP(hipMemcpyAsync(&P->n_pairs, part_base + n_part, 8, hipMemcpyDeviceToHost, st));
    LDDL_HIP(hipStreamSynchronize(st));
    max_np = std::max<int64_t>(1, (int64_t)ctl[3]);
    if (!prm->masking) break;
    if (!ctl[1]) {
      P->mtok = mtok;
      TRY(P->alloc(&P->mpos, (int64_t)ctl[0], st));
      break;
    }
    P->free_one(mtok, st);
    P->free_one(jpool, st);
    jpool = nullptr;
    if (attempt > 0) TRY((set_error("mask pool overflow after resize"), -1));
    cap = (int64_t)ctl[0] + 1024;
    jcap = (int64_t)ctl[2] + 1024;
  }
  // the pair maps (see PairMaps): with masking the planner-order slots and their output
  // positions (the mask replay writes each pair's gather record there), else the output order
  PairMaps M{part_base, nullptr, nullptr, nullptr};
  if (prm->masking) {
    TRY(P->alloc(&M.slots, P->n_pairs, st));
    TRY(P->alloc(&M.dstq, P->n_pairs, st));
  } else {
    TRY(P->alloc(&P->src, P->n_pairs, st));
    M.src = P->src;
  }
  // random.shuffle(partition_pairs), alone on the stream (its blocks need 16 waves and ~90 KB of
  // LDS per CU: beside fy_resolve's small blocks on a second stream they waited for CUs to
  // drain, 10.3 ms against ~2 alone); its last pass writes the pair maps
  if (n_part) {
    const int64_t cap = max_np;
    // dynamic-LDS budget of the swap kernel: what the device grants a block (160 KiB on
    // gfx950), minus headroom for the kernel's static LDS
    const size_t kLdsBudget = std::min<size_t>(150 * 1024, c->lds_per_block > 10 * 1024
                                                               ? c->lds_per_block - 10 * 1024 : 0);
    const bool force_global = getenv("LDDL_SHUFFLE_GLOBAL") != nullptr;  // tests: the large-partition path
    // partitions of <= cap_lds pairs: the parallel bucket-sort resolve (three 16-bit LDS tables);
    // larger ones: one lane swapping in global memory
    const int64_t cap_lds = force_global ? 0 : std::min<int64_t>({cap, 65534, (int64_t)(kLdsBudget / 6) - 2});
    if (cap_lds > 0)
      hipLaunchKernelGGL(shuffle_sort_kernel, dim3((unsigned)n_part), dim3(kShufThreads),
                         (size_t)6 * (size_t)((cap_lds + 2) & ~1), st, P->kd_off, P->kp_off,
                         prm->dup, part_npairs, jseq, P->order, (int32_t)cap_lds, M);
    if (cap > cap_lds) {  // partitions beyond the LDS tables: swaps in global memory, then the maps
      hipLaunchKernelGGL(apply_shuffle_kernel, dim3((unsigned)n_part), dim3(64), 0, st, P->kd_off,
                         P->kp_off, prm->dup, part_npairs, jseq, P->order, cap_lds);
      hipLaunchKernelGGL(map_pairs_kernel, dim3((unsigned)n_part), dim3(256), 0, st, P->kd_off,
                         P->kp_off, prm->dup, part_base, (const int32_t*)P->order, M.src, M.slots,
                         M.dstq);
    }
  }
  LDDL_HIP(hipGetLastError());
#ifdef LDDL_STAMPS
  {
    std::vector<uint64_t> h(n_part * kStampRegions);
    LDDL_HIP(hipMemcpyAsync(h.data(), d_stamps, 8 * h.size(), hipMemcpyDeviceToHost, st));
    LDDL_HIP(hipStreamSynchronize(st));
    double tot[kStampRegions] = {0};
    for (int64_t q = 0; q < n_part; ++q)
      for (int r = 0; r < kStampRegions; ++r) tot[r] += (double)h[q * kStampRegions + r];
    const char* names[kStampRegions] = {"plan", "cand", "shuffle_draws", "random_next", "decisions",
                                        "trunc", "final_shuffle_draws", "fy_jacobi_passes_per_window"};
    double all = 0;
    for (int r = 0; r < kStampRegions - 1; ++r) all += tot[r];
    fprintf(stderr, "[stamps] plan_replay_kernel mean cycles per partition:");
    for (int r = 0; r < kStampRegions - 1; ++r)
      fprintf(stderr, " %s=%.3g (%.1f%%)", names[r], tot[r] / n_part, 100.0 * tot[r] / (all + 1e-9));
    fprintf(stderr, " %s=%.3f\n", names[kStampRegions - 1], tot[kStampRegions - 1] / n_part / 1e6);
    // timeline (100 MHz real-time clock): partition durations and concurrency over the launch
    std::vector<uint64_t> t(2 * n_part);
    LDDL_HIP(hipMemcpyAsync(t.data(), d_tl, 16 * n_part, hipMemcpyDeviceToHost, st));
    LDDL_HIP(hipStreamSynchronize(st));
    uint64_t t0 = ~0ull, t1 = 0;
    std::vector<double> dur(n_part);
    for (int64_t q = 0; q < n_part; ++q) {
      t0 = std::min(t0, t[2 * q]);
      t1 = std::max(t1, t[2 * q + 1]);
      dur[q] = (t[2 * q + 1] - t[2 * q]) / 1e5;  // ms
    }
    std::vector<double> sd = dur;
    std::sort(sd.begin(), sd.end());
    const double span = (t1 - t0) / 1e5;
    fprintf(stderr, "[timeline] span %.2f ms, partition ms min %.2f p10 %.2f p50 %.2f p90 %.2f max %.2f\n",
            span, sd[0], sd[n_part / 10], sd[n_part / 2], sd[n_part * 9 / 10], sd[n_part - 1]);
    const int nb = 40;
    fprintf(stderr, "[timeline] active partitions per %.2f ms bin:", span / nb);
    for (int b = 0; b < nb; ++b) {
      const uint64_t a = t0 + (t1 - t0) * b / nb, e = t0 + (t1 - t0) * (b + 1) / nb;
      double act = 0;  // partition-time inside the bin / bin length
      for (int64_t q = 0; q < n_part; ++q) {
        const uint64_t s0 = std::max(a, t[2 * q]), s1 = std::min(e, t[2 * q + 1]);
        if (s1 > s0) act += (double)(s1 - s0);
      }
      fprintf(stderr, " %.0f", act / (double)(e - a));
    }
    fprintf(stderr, "\n[timeline] start ms of partitions by index decile:");
    for (int k = 0; k <= 10; ++k) {
      const int64_t q = std::min<int64_t>(n_part - 1, n_part * k / 10);
      fprintf(stderr, " %.1f", (t[2 * q] - t0) / 1e5);
    }
    fprintf(stderr, "\n");
  }
#endif
  // layout (part_base and n_pairs came with the planner's sync). With masking, the mask replay
  // (fy_resolve, planner order) also writes every pair's gather record at its output position
  // and the two output-order scans follow; without, pair_prep builds the records from the
  // output order. (Round 4 ran pair_prep beside fy_resolve on a second stream: 15.6 ms for the
  // section, both kernels slowed by the other; the fused replay reads each slot record once.)
  TRY(alloc_layout(P->n_pairs));
  if (prm->masking) {
    if (P->n_pairs) {
      ResolveArgs RA{M.slots, P->n_pairs, P->desc, spool, jpool, P->mpos, P->kscan, P->dense, cls,
                     sep, M.dstq, P->rec, pcnt, 0};
      const dim3 grid((unsigned)((P->n_pairs + 63) / 64));
      // a lane's column covers the padded draw region (steps up to nc rounded up to 16)
      const size_t col = (size_t)((prm->seq + 15) & ~15);
      RA.col_rows = (int32_t)col;
      // Branch-free steps for long pairs (C3, seq 512: 77.6 -> 46.8 ms), the guarded ones at
      // seq <= 131 (64 pairs per wave: 10.1 ms against 11.5 branch-free; profiles/r05k_*).
      // A/B: LDDL_FY_MODE=0 / 1 forces one kind everywhere; LDDL_FY_LW=32: 32 pairs per wave at
      // seq > 256 (50.7 ms)
      const int fy_mode = getenv("LDDL_FY_MODE") ? atoi(getenv("LDDL_FY_MODE")) : -1;
      const int fy_lw = getenv("LDDL_FY_LW") ? atoi(getenv("LDDL_FY_LW")) : 16;
      // move-only groups at seq > 256 read one entry ahead (46.8 -> 44.4 ms; 2 ahead 45.9, 3 ahead
      // 46.7: the forwarding selects grow; profiles/r05m_*). LDDL_FY_RA=0..3 (A/B)
      const int fy_ra = getenv("LDDL_FY_RA") ? atoi(getenv("LDDL_FY_RA")) : 1;
      // draw vectors (8 steps each) in flight per lane at seq > 256 (A/B: LDDL_FY_PF=2 / 8)
      const int fy_pf = getenv("LDDL_FY_PF") ? atoi(getenv("LDDL_FY_PF")) : 4;
      // the A/B knobs take only the values a test runs (unsupported values and
      // combinations were ignored without notice)
      if (fy_mode < -1 || fy_mode > 1) LDDL_FAIL(-1, "LDDL_FY_MODE must be 0 or 1");
      if (fy_lw != 16 && fy_lw != 32) LDDL_FAIL(-1, "LDDL_FY_LW must be 16 or 32");
      if (fy_ra < 0 || fy_ra > 3) LDDL_FAIL(-1, "LDDL_FY_RA must be 0 .. 3");
      if (fy_pf != 2 && fy_pf != 4 && fy_pf != 8) LDDL_FAIL(-1, "LDDL_FY_PF must be 2, 4 or 8");
      if (fy_pf != 4 && fy_ra != 1) LDDL_FAIL(-1, "LDDL_FY_PF applies with LDDL_FY_RA=1 only");
      if ((fy_ra != 1 || fy_pf != 4) && (fy_mode == 0 || fy_lw == 32))
        LDDL_FAIL(-1, "LDDL_FY_RA / PF select 16-lane branch-free variants (not with LDDL_FY_MODE=0 "
                      "or LDDL_FY_LW=32)");
#define LDDL_FY_LAUNCH(T, NG, LW, BF, ...)                                                     \
  hipLaunchKernelGGL((fy_resolve_kernel<T, T, NG, LW, BF, ##__VA_ARGS__>),                     \
                     dim3((unsigned)((P->n_pairs + LW - 1) / LW)), dim3(LW),                   \
                     (size_t)LW * sizeof(T) * col, st, RA)
      if (prm->seq <= 131) {  // nc <= 128: all draws in registers (8 uint4 of 1-byte draws); 64
        // pairs per wave (C2: 10.2 ms; 32 per wave 11.9, 16 per wave 20.1, profiles/r04slw_*)
        if (fy_mode == 1) LDDL_FY_LAUNCH(uint8_t, 8, 64, true);
        else LDDL_FY_LAUNCH(uint8_t, 8, 64, false);
      // long pairs: 16 lanes (pairs) per wave (C3, seq 512: 106 ms with 64, 109 with 32, 93 with
      // 16; profiles/r04fy_*)
      } else if (prm->seq <= 256) {  // candidate indices, positions and draws fit a byte
        if (fy_mode) LDDL_FY_LAUNCH(uint8_t, 0, 16, true);
        else LDDL_FY_LAUNCH(uint8_t, 0, 16, false);
      } else if (fy_lw == 32) {
        if (fy_mode) LDDL_FY_LAUNCH(uint16_t, 0, 32, true);
        else LDDL_FY_LAUNCH(uint16_t, 0, 32, false);
      } else {
        if (!fy_mode) LDDL_FY_LAUNCH(uint16_t, 0, 16, false);
        else if (fy_ra == 1 && fy_pf == 8) LDDL_FY_LAUNCH(uint16_t, 0, 16, true, 1, 8);
        else if (fy_ra == 1 && fy_pf == 2) LDDL_FY_LAUNCH(uint16_t, 0, 16, true, 1, 2);
        else if (fy_ra == 1) LDDL_FY_LAUNCH(uint16_t, 0, 16, true, 1);
        else if (fy_ra == 2) LDDL_FY_LAUNCH(uint16_t, 0, 16, true, 2);
        else if (fy_ra == 3) LDDL_FY_LAUNCH(uint16_t, 0, 16, true, 3);
        else LDDL_FY_LAUNCH(uint16_t, 0, 16, true);
      }
#undef LDDL_FY_LAUNCH
    }
    LDDL_HIP(hipGetLastError());
    TRY(scan_only(st));
  } else {
    TRY(prep_and_scan(st));
  }
  }  // replay
  if (prm->rng == LDDL_RNG_NATIVE) {
    TRY(alloc_layout(P->n_pairs));
    TRY(prep_and_scan(st));
  }
  LDDL_HIP(hipMemcpyAsync(&P->n_tokens, P->tok_off + P->n_pairs, 8, hipMemcpyDeviceToHost, st));
  if (prm->masking)
    LDDL_HIP(hipMemcpyAsync(&P->n_masked, P->pos_off + P->n_pairs, 8, hipMemcpyDeviceToHost, st));
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

extern "C" int lddl_pairs_emit(lddl_pairs* P, void* stream, void* d_tokens, int64_t* d_tok_off,
                               int32_t* d_len_a, uint8_t* d_is_rn, uint16_t* d_pos, void* d_lab,
                               int64_t* d_pos_off) {
  if (!P) LDDL_FAIL(-1, "null plan");
  hipStream_t st = as_stream(stream);
  if (P->n_pairs == 0) return 0;
  GatherArgs G{};
  G.dense = P->dense.p;
  G.rec = P->rec;
  G.mpos = P->mpos;
  G.mtok = P->mtok;
  G.masking = P->masking;
  G.n_pairs = P->n_pairs;
  G.tok_off = P->tok_off;
  G.pos_off = P->pos_off;
  G.out_tok = d_tokens;
  G.len_a = d_len_a;
  G.is_rn = d_is_rn;
  G.out_pos = d_pos;
  G.out_lab = d_lab;
  G.out_tok_off = d_tok_off;
  G.out_pos_off = d_pos_off;
  GatherLds Lg{(P->seq + 127) / 128 * 128, P->dense.ib, P->dense.ib == 2 && P->seq <= 600 ? 2 : 4};
  auto launch = [&](auto kern, int K) {
    const int64_t per_wg = (int64_t)2 * K * kGWaves;
    const int64_t nwg = (P->n_pairs + per_wg - 1) / per_wg;
    const int64_t gx = std::min<int64_t>(nwg, 65536);
    const size_t lds = P->masking ? (size_t)kGWaves * 2 * K * Lg.per_pair() : 0;
    hipLaunchKernelGGL(kern, dim3((unsigned)gx, (unsigned)((nwg + gx - 1) / gx)), dim3(64 * kGWaves),
                       lds, st, G, Lg);
  };
  const bool i16 = P->dense.ib == 2;
  if (P->seq <= 600) {
    if (i16) launch(gather16_kernel<16>, 2);  // (4 pairs per wave, like K = 2; LP = 8: 35.3 ms, r04ze)
    else launch(gather_kernel<2, int32_t>, 2);
  } else {  // (LDS: seq-entry decision tables)
    if (i16) launch(gather_kernel<1, uint16_t>, 1);
    else launch(gather_kernel<1, int32_t>, 1);
  }
  LDDL_HIP(hipGetLastError());
  return 0;
}

extern "C" int lddl_pairs_destroy(lddl_pairs* P, void* stream) {
  if (!P) return 0;
  P->release(as_stream(stream));
  delete P;
  return 0;
}

extern "C" int lddl_pairs_plan_ms(const lddl_pairs* P, float* ms) {
  if (!P || !ms) LDDL_FAIL(-1, "null argument");
  *ms = 0.f;
  if (P->n_part && P->ev[0]) LDDL_HIP(hipEventElapsedTime(ms, P->ev[0], P->ev[1]));
  return 0;
}

extern "C" int lddl_pairs_part_offsets(lddl_pairs* P, void* stream, int64_t* d_part_pair_off) {
  if (!P || !d_part_pair_off) LDDL_FAIL(-1, "null argument");
  LDDL_HIP(hipMemcpyAsync(d_part_pair_off, P->part_base, 8 * (P->n_part + 1),
                          hipMemcpyDeviceToDevice, as_stream(stream)));
  return 0;
}
