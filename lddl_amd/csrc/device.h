// Device-side shared definitions: context tables, vocab hash, wave primitives.
#pragma once
#include <type_traits>
#include <hip/hip_runtime.h>
#include <cstdint>

namespace lddl {

// ---- vocab hash entry (16 B): exact key for pieces <= 12 bytes, prefix + tail check beyond ----
// meta: bit31 valid | bit30 continuation ("##") | bit29 long (len > 12) | bits 28..21 len |
//       bits 20..0 id
struct alignas(16) VEnt {
  uint64_t k0;
  uint32_t k1;
  uint32_t meta;
};

constexpr uint32_t kMetaValid = 1u << 31, kMetaCont = 1u << 30, kMetaLong = 1u << 29;

__host__ __device__ inline uint32_t meta_len(uint32_t m) { return (m >> 21) & 0xFF; }
__host__ __device__ inline int32_t meta_id(uint32_t m) { return (int32_t)(m & 0x1FFFFF); }

__host__ __device__ inline uint64_t vhash(uint64_t k0, uint32_t k1, uint32_t len, uint32_t cont) {
  // 32-bit multiplies only (v_mul_lo_u32): a 64-bit multiply costs ~4 of them on CDNA
  uint32_t h = (uint32_t)k0 * 0x9E3779B1u;
  h ^= ((uint32_t)(k0 >> 32) + (len << 24) + cont) * 0x85EBCA77u;
  h ^= k1 * 0xC2B2AE3Du;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 13;
  return h;
}

// keep the low `len` bytes of a little-endian packed word (len in 0..8)
__host__ __device__ inline uint64_t keep_bytes(uint64_t v, int len) {
  return len >= 8 ? v : (len <= 0 ? 0 : (v & ((1ull << (8 * len)) - 1)));
}

// ---- normaliser table classes (tools/make_norm_tables.py) ----
constexpr uint32_t kWord = 0, kDrop = 1, kSpace = 2, kIso = 3;
constexpr uint32_t kIdent = 1u << 29, kMulti = 1u << 28;

// Special tokens matched on raw text (added tokens, normalized=False), fixed order.
constexpr int kNumSpecial = 5;  // [PAD] [UNK] [CLS] [SEP] [MASK]
enum { kPad = 0, kUnk = 1, kCls = 2, kSep = 3, kMask = 4 };

// Kernel-side view of a context (passed by value).
struct Tables {
  const uint16_t* l1;
  const uint32_t* pages;
  const uint8_t* pool;
  const VEnt* vhash;
  const uint8_t* vbytes;  // piece bytes without "##", piece i at vbytes[voff[i]..voff[i+1])
  const int64_t* voff;
  uint32_t vmask;
  int32_t max_piece_bytes;
  int32_t special_id[kNumSpecial];
  // ASCII fast path of the wave tokenizer: 1 = ASCII WORD chars map to themselves except A-Z ->
  // a-z (uncased table), 2 = all map to themselves (cased), 0 = neither (fast path disabled)
  int32_t ascii_mode;
  const uint32_t* bloom;  // kBloomWords words: Bloom filter of (continuation, piece bytes)
  // piece i's first 32 bytes, zero-padded, at vlong[4 i .. 4 i + 4): the tail check of a hash hit
  // on a piece longer than the 12-byte key, as three masked 64-bit compares
  const uint64_t* vlong;
};

// Bloom filter over vocab pieces for the longest-match scan: a piece's prefix hash is a
// polynomial over its bytes (h = h * P + b + 1 mod 2^32, so every prefix of a word comes from one
// pass), mixed with its length and continuation flag; two bits in one 32-bit word.
constexpr int kBloomWords = 8192;  // 32 KB
constexpr uint32_t kBloomP = 0x01000193u;
// One multiply: the word index comes from the top 13 bits of the product and the two bit
// positions from its middle bits (the prefix hash h is already well mixed; in the longest-match
// scan this runs once per candidate length, so it is kept short).
__host__ __device__ inline uint32_t bloom_mix(uint32_t h, uint32_t len, uint32_t cont) {
  return (h ^ (len << 24) ^ (cont << 31)) * 0x85EBCA6Bu;
}
__host__ __device__ inline uint32_t bloom_word(uint32_t x) { return x >> 19; }
__host__ __device__ inline uint32_t bloom_bits(uint32_t x) {
  return (1u << ((x >> 9) & 31u)) | (1u << ((x >> 14) & 31u));
}

// sent_len flag: the kept pieces contain a literal [CLS] or [SEP] (matters for static masking
// candidates, pretrain.py:189-192)
constexpr int32_t kLenHasClsSep = 1 << 30;
constexpr int32_t kLenMask = (1 << 30) - 1;

// ---- wave helpers (wave64) ----
__device__ inline int lane_id() { return __lane_id(); }
// the wave's index in its workgroup as a wave-uniform value: the compiler treats threadIdx.x >> 6 as
// divergent, and indices derived from it turned loop bounds and early exits into exec-mask code
// (tokenizer: 14.78 -> 14.39 ms per 2 GB, profiles/r06tk2_tok_uniform_chunk_ab.txt)
__device__ inline int wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }

// Inclusive prefix sum over the 64 lanes (all lanes active) with DPP: row_shr 1/2/4/8 sums
// within each 16-lane row, then row_bcast:15 and row_bcast:31 carry the row totals (GFX9 DPP).
// Six VALU ops with DPP source modifiers per 32-bit half; no LDS traffic, no lane masks.
template <int kCtrl, int kRowMask, bool kBound>
__device__ inline uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, kRowMask, 0xF, kBound);
}
template <int kCtrl, int kRowMask, bool kBound>
__device__ inline uint32_t scan_step(uint32_t v) {
  return v + dpp_u32<kCtrl, kRowMask, kBound>(v);
}
template <int kCtrl, int kRowMask, bool kBound>
__device__ inline uint64_t scan_step(uint64_t v) {
  const uint32_t lo = dpp_u32<kCtrl, kRowMask, kBound>((uint32_t)v);
  const uint32_t hi = dpp_u32<kCtrl, kRowMask, kBound>((uint32_t)(v >> 32));
  return v + (((uint64_t)hi << 32) | lo);
}
// v of lane l - 1 (lane 0: its own v) / of lane l + 1 (lane 63: its own v): whole-wave DPP shifts
__device__ inline int wave_prev(int v) { return __builtin_amdgcn_update_dpp(v, v, 0x138, 0xF, 0xF, false); }
__device__ inline int wave_next(int v) { return __builtin_amdgcn_update_dpp(v, v, 0x130, 0xF, 0xF, false); }

template <typename T>
__device__ inline T wave_incl_scan(T v) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "32- or 64-bit scan");
  using U = std::conditional_t<sizeof(T) == 4, uint32_t, uint64_t>;
  U u = (U)v;
  u = scan_step<0x111, 0xF, true>(u);   // row_shr:1
  u = scan_step<0x112, 0xF, true>(u);   // row_shr:2
  u = scan_step<0x114, 0xF, true>(u);   // row_shr:4
  u = scan_step<0x118, 0xF, true>(u);   // row_shr:8
  u = scan_step<0x142, 0xA, false>(u);  // row_bcast:15 -> rows 1, 3
  u = scan_step<0x143, 0xC, false>(u);  // row_bcast:31 -> rows 2, 3
  return (T)u;
}

// Philox4x32-10 (Salmon et al., SC'11)
struct Philox {
  __device__ static uint4 round(uint4 c, uint2 k) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    return make_uint4((uint32_t)(p1 >> 32) ^ c.y ^ k.x, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k.y,
                      (uint32_t)p0);
  }
  __device__ static uint4 gen(uint4 c, uint2 k) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      c = round(c, k);
      k.x += 0x9E3779B9u;
      k.y += 0xBB67AE85u;
    }
    return c;
  }
};

// Lane mask of a predicate. The bool overload lets the compiler use the condition's lane mask
// directly (HIP's __ballot(int) re-materialises it through a compare against zero).
__device__ inline uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// Workgroup b of a launch of nb as the logical block that keeps each XCD's share contiguous:
// the dispatcher deals workgroups round-robin over the 8 XCDs (b and b + 8 share one XCD and its
// L2; MI355X_MICROARCH.md, workgroup dispatch), so consecutive logical blocks - e.g. the pairs
// of one partition, which re-read the same dense tokens and mask pool lines - meet in one L2
// instead of eight. A bijection on [0, nb); placement only, never correctness.
__device__ inline int64_t xcd_block(int64_t b, int64_t nb) {
  const int64_t per = nb >> 3, rem = nb & 7, x = b & 7;
  return x * per + (x < rem ? x : rem) + (b >> 3);
}

// Set bits of m below the calling lane (v_mbcnt).
__device__ inline uint32_t popc_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// LDS written by some lanes of a wave becomes visible to all lanes of that wave
__device__ inline void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <typename T>
__device__ inline T wave_sum(T v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

}  // namespace lddl
