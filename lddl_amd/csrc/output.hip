// Sample table -> output layout on the GPU: per-partition sequence-length binning and the string /
// npy rendering of the parquet columns.
//
// Reference:
//   _to_dataframe_binned           lddl/dask/bert/binning.py:63-93   -> bin_partitions_kernel
//     bin_id = min((num_tokens - 1) // bin_size, nbins - 1); rows of a partition regrouped by bin,
//     stable within a bin (pd.concat of per-bin frames in bin order).
//   instance dict                  lddl/dask/bert/pretrain.py:345-358 -> render_*_kernel
//     A / B = ' '.join(tokens), masked_lm_labels = ' '.join(labels),
//     masked_lm_positions = serialize_np_array(uint16[k]) (lddl/utils.py:98-102: np.save bytes,
//     a fixed 128-byte v1.0 header then 2k little-endian bytes).
//
// bin_partitions_kernel: one workgroup per partition. Pass 1 counts rows per bin in LDS; an LDS
// scan turns counts into bin bases; pass 2 walks the partition in order 64 rows at a time and
// ranks each row among earlier rows of the same bin: running per-bin counter (LDS) + the lanes
// below it with the same bin, found with bit-sliced ballots (one ballot per bit of the bin id).
// Only wave 0 runs pass 2, so the per-bin counters need no atomics and order is preserved.
//
// render: one wavefront per row. Lane j owns token j of a 64-token chunk; its string length
// comes from the vocab render table, a wave scan gives byte offsets, and each lane copies its
// token string and the separating space.
#include <algorithm>
#include <cstring>

#include "common.h"
#include "ctx.h"
#include "device.h"
#include "lddl_amd.h"
#include "scan.h"

namespace lddl {
namespace {

constexpr int kBinThreads = 256;
constexpr int kMaxBinsLds = 8192;

__device__ inline int32_t bin_of(int32_t nt, int32_t bin_size, int32_t nbins) {
  const int32_t b = (nt - 1) / bin_size;  // num_tokens >= 5 (>= 1 token in A and in B)
  return b > nbins - 1 ? nbins - 1 : b;
}

// num_tokens of row r: an int32 column, or (tok_off given) the pair's token count + 3
struct NumTok {
  const int32_t* nt;
  const int64_t* tok_off;
  __device__ int32_t operator[](int64_t r) const {
    return nt ? nt[r] : (int32_t)(tok_off[r + 1] - tok_off[r] + 3);
  }
};

__global__ void __launch_bounds__(kBinThreads) bin_partitions_kernel(
    NumTok num_tokens, const int64_t* __restrict__ part_off, int32_t bin_size,
    int32_t nbins, int32_t nbits, int64_t* __restrict__ perm, int64_t* __restrict__ bin_id,
    int64_t* __restrict__ counts) {
  __shared__ int64_t s_cnt[kMaxBinsLds];
  __shared__ int64_t s_tot[kBinThreads / 64];
  const int64_t p = blockIdx.x;
  const int64_t r0 = part_off[p], r1 = part_off[p + 1];
  for (int b = threadIdx.x; b < nbins; b += kBinThreads) s_cnt[b] = 0;
  __syncthreads();
  for (int64_t r = r0 + threadIdx.x; r < r1; r += kBinThreads)
    atomicAdd(reinterpret_cast<unsigned long long*>(&s_cnt[bin_of(num_tokens[r], bin_size, nbins)]),
              1ull);
  __syncthreads();
  // counts out, then exclusive scan of s_cnt in place (bins in chunks of kBinThreads)
  for (int b = threadIdx.x; b < nbins; b += kBinThreads) counts[p * nbins + b] = s_cnt[b];
  int64_t carry = 0;
  for (int b0 = 0; b0 < nbins; b0 += kBinThreads) {
    const int b = b0 + threadIdx.x;
    const int64_t v = b < nbins ? s_cnt[b] : 0;
    const int64_t incl = wave_incl_scan(v);
    if (lane_id() == 63) s_tot[threadIdx.x >> 6] = incl;
    __syncthreads();
    int64_t off = carry;
    int64_t tot = 0;
    for (int w = 0; w < kBinThreads / 64; ++w) {
      if (w < (int)(threadIdx.x >> 6)) off += s_tot[w];
      tot += s_tot[w];
    }
    __syncthreads();
    if (b < nbins) s_cnt[b] = off + incl - v;
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  const uint64_t below = (1ull << lane) - 1;
  for (int64_t c0 = r0; c0 < r1; c0 += 64) {
    const int64_t r = c0 + lane;
    const bool in = r < r1;
    const int32_t b = in ? bin_of(num_tokens[r], bin_size, nbins) : -1;
    uint64_t match = ballot(in);
    for (int k = 0; k < nbits; ++k) {
      const uint64_t bk = ballot(in && ((b >> k) & 1));
      match &= ((b >> k) & 1) ? bk : ~bk;
    }
    const int rank = (int)popc_below(match);
    int64_t base = 0;
    if (in) base = s_cnt[b];
    __builtin_amdgcn_wave_barrier();
    if (in) {
      const int64_t dst = r0 + base + rank;
      perm[dst] = r;
      bin_id[dst] = b;
      if ((match & below) == 0) s_cnt[b] = base + __popcll(match);  // group leader advances
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}


// ---- stable sort by bin of one large segment: tiles of kBinTile rows, one wavefront each ----
constexpr int kBinTile = 2048;


__global__ void __launch_bounds__(64) bin_tile_hist_kernel(NumTok num_tokens,
                                                           int64_t n, int32_t bin_size,
                                                           int32_t nbins, int64_t n_tiles,
                                                           int64_t* __restrict__ tile_counts) {
  __shared__ int32_t s_cnt[kMaxBinsLds];
  const int64_t tile = blockIdx.x;
  for (int b = threadIdx.x; b < nbins; b += 64) s_cnt[b] = 0;
  __syncthreads();
  const int64_t r0 = tile * kBinTile, r1 = min(n, r0 + kBinTile);
  for (int64_t r = r0 + threadIdx.x; r < r1; r += 64)
    atomicAdd(&s_cnt[bin_of(num_tokens[r], bin_size, nbins)], 1);
  __syncthreads();
  for (int b = threadIdx.x; b < nbins; b += 64) tile_counts[(int64_t)b * n_tiles + tile] = s_cnt[b];
}

__global__ void __launch_bounds__(64) bin_tile_scatter_kernel(
    NumTok num_tokens, int64_t n, int32_t bin_size, int32_t nbins,
    int32_t nbits, int64_t n_tiles, const int64_t* __restrict__ tile_base,
    int64_t* __restrict__ perm, int64_t* __restrict__ bin_id) {
  __shared__ int64_t s_run[kMaxBinsLds];
  const int64_t tile = blockIdx.x;
  for (int b = threadIdx.x; b < nbins; b += 64) s_run[b] = tile_base[(int64_t)b * n_tiles + tile];
  __syncthreads();
  const int lane = threadIdx.x;
  const uint64_t below = (1ull << lane) - 1;
  const int64_t r0 = tile * kBinTile, r1 = min(n, r0 + kBinTile);
  for (int64_t c0 = r0; c0 < r1; c0 += 64) {
    const int64_t r = c0 + lane;
    const bool in = r < r1;
    const int32_t b = in ? bin_of(num_tokens[r], bin_size, nbins) : -1;
    uint64_t match = ballot(in);
    for (int k = 0; k < nbits; ++k) {
      const uint64_t bk = ballot(in && ((b >> k) & 1));
      match &= ((b >> k) & 1) ? bk : ~bk;
    }
    int64_t base = 0;
    if (in) base = s_run[b];
    __builtin_amdgcn_wave_barrier();
    if (in) {
      const int64_t dst = base + (int)popc_below(match);
      perm[dst] = r;
      if (bin_id) bin_id[dst] = b;
      if ((match & below) == 0) s_run[b] = base + __popcll(match);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// bin totals = column sums of the tile counts (bin b's tiles are contiguous after the scan)
__global__ void bin_totals_kernel(const int64_t* __restrict__ tile_base, int64_t n_tiles,
                                  int32_t nbins, int64_t* __restrict__ counts) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < nbins) counts[b] = tile_base[(int64_t)(b + 1) * n_tiles] - tile_base[(int64_t)b * n_tiles];
}

// ---- rendering --------------------------------------------------------------------------------
struct RenderArgs {
  const uint8_t* rbytes;  // vocab render table
  const int64_t* roff;
  const void* tokens;  // ids of lddl_ctx::id_bytes bytes each (uint16 or int32)
  const int64_t* tok_off;
  const int32_t* len_a;
  const uint16_t* pos;
  const void* lab;     // as tokens
  const int64_t* pos_off;
  const int64_t* rows;  // output row -> pair (NULL: identity)
  int64_t n_rows;
  int32_t ib;           // bytes per id
};

// id i of an id array of R.ib-byte entries
__device__ inline int32_t id_at(const RenderArgs& R, const void* ids, int64_t i) {
  return R.ib == 2 ? (int32_t)static_cast<const uint16_t*>(ids)[i] : static_cast<const int32_t*>(ids)[i];
}

__device__ inline int32_t tok_len(const RenderArgs& R, int32_t id) {
  return (int32_t)(R.roff[id + 1] - R.roff[id]);
}

// total bytes of ' '.join(strings of ids[i0 .. i0 + n))
__device__ int64_t joined_len(const RenderArgs& R, const void* ids, int64_t i0, int64_t n) {
  int64_t acc = 0;
  for (int64_t c0 = 0; c0 < n; c0 += 64) {
    const int64_t j = c0 + lane_id();
    acc += j < n ? tok_len(R, id_at(R, ids, i0 + j)) : 0;
  }
  return wave_sum(acc) + (n > 0 ? n - 1 : 0);
}

__device__ void joined_write(const RenderArgs& R, const void* ids, int64_t i0, int64_t n,
                             uint8_t* out) {
  int64_t base = 0;
  for (int64_t c0 = 0; c0 < n; c0 += 64) {
    const int64_t j = c0 + lane_id();
    const int32_t id = j < n ? id_at(R, ids, i0 + j) : 0;
    const int64_t l = j < n ? tok_len(R, id) + 1 : 0;  // string + separator
    const int64_t incl = wave_incl_scan(l);
    if (j < n) {
      uint8_t* o = out + base + incl - l;
      const uint8_t* src = R.rbytes + R.roff[id];
      for (int64_t q = 0; q < l - 1; ++q) o[q] = src[q];
      if (j < n - 1) o[l - 1] = ' ';
    }
    base += __shfl(incl, 63, 64);
  }
}

__global__ void __launch_bounds__(256) render_lengths_kernel(RenderArgs R, int64_t* a_len,
                                                             int64_t* b_len, int64_t* l_len,
                                                             int64_t* n_pos, const uint8_t* is_rn,
                                                             uint16_t* num_tokens_out,
                                                             uint8_t* is_rn_out) {
  const int64_t row = (int64_t)blockIdx.x * 4 + wave_id();
  if (row >= R.n_rows) return;
  const int64_t q = R.rows ? R.rows[row] : row;
  const int64_t t0 = R.tok_off[q], t1 = R.tok_off[q + 1];
  const int32_t na = R.len_a[q];
  const int64_t la = joined_len(R, R.tokens, t0, na);
  const int64_t lb = joined_len(R, R.tokens, t0 + na, t1 - t0 - na);
  int64_t ll = 0, np = 0;
  if (R.pos_off) {
    const int64_t p0 = R.pos_off[q], p1 = R.pos_off[q + 1];
    ll = joined_len(R, R.lab, p0, p1 - p0);
    np = p1 - p0;
  }
  if (lane_id() == 0) {
    a_len[row] = la;
    b_len[row] = lb;
    if (l_len) l_len[row] = ll;
    if (n_pos) n_pos[row] = 128 + 2 * np;
    // the row's num_tokens / is_random_next columns in output order
    if (num_tokens_out) num_tokens_out[row] = (uint16_t)(t1 - t0 + 3);
    if (is_rn_out) is_rn_out[row] = is_rn[q];
  }
}

__device__ void put_npy(uint8_t* o, const uint16_t* pos, int64_t k) {
  // 128-byte NPY v1.0 header of a 1-D '<u2' array of length k, as np.save writes it
  const char* pre = "\x93NUMPY\x01\x00v\x00{'descr': '<u2', 'fortran_order': False, 'shape': (";
  const int pre_len = 10 + 51;
  char digits[24];
  int nd = 0;
  int64_t v = k;
  do { digits[nd++] = (char)('0' + v % 10); v /= 10; } while (v);
  const int lane = lane_id();
  for (int i = lane; i < 128; i += 64) {
    char c;
    if (i < pre_len) c = pre[i];
    else if (i < pre_len + nd) c = digits[nd - 1 - (i - pre_len)];
    else if (i < pre_len + nd + 5) c = ",), }"[i - pre_len - nd];
    else if (i < 127) c = ' ';
    else c = '\n';
    o[i] = (uint8_t)c;
  }
  for (int64_t j = lane; j < k; j += 64) {
    o[128 + 2 * j] = (uint8_t)(pos[j] & 0xFF);
    o[128 + 2 * j + 1] = (uint8_t)(pos[j] >> 8);
  }
}

__global__ void __launch_bounds__(256) render_write_kernel(RenderArgs R, const int64_t* a_off,
                                                           const int64_t* b_off, const int64_t* l_off,
                                                           const int64_t* npy_off, uint8_t* a_bytes,
                                                           uint8_t* b_bytes, uint8_t* l_bytes,
                                                           uint8_t* npy_bytes) {
  const int64_t row = (int64_t)blockIdx.x * 4 + wave_id();
  if (row >= R.n_rows) return;
  const int64_t q = R.rows ? R.rows[row] : row;
  const int64_t t0 = R.tok_off[q], t1 = R.tok_off[q + 1];
  const int32_t na = R.len_a[q];
  joined_write(R, R.tokens, t0, na, a_bytes + a_off[row]);
  joined_write(R, R.tokens, t0 + na, t1 - t0 - na, b_bytes + b_off[row]);
  if (R.pos_off) {
    const int64_t p0 = R.pos_off[q], p1 = R.pos_off[q + 1];
    if (l_bytes) joined_write(R, R.lab, p0, p1 - p0, l_bytes + l_off[row]);
    if (npy_bytes) put_npy(npy_bytes + npy_off[row], R.pos + p0, p1 - p0);
  }
}

// ---- row movement of the load balance (lddl_amd/balance.py) ----------------------------------
// Rows are addressed over two sources: row r < n_a is row r of source A, else row r - n_a of
// source B (a rank's own table and the rows it received), so the exchange never concatenates.
template <typename T>
struct Src2 {
  const T* a;
  const T* b;
  int64_t n_a;
  __device__ const T* at(int64_t r) const { return r < n_a ? a + r : b + (r - n_a); }
};

template <typename T>
__global__ void __launch_bounds__(256) gather_ragged_kernel(Src2<T> src, Src2<int64_t> off,
                                                            const int64_t* __restrict__ rows,
                                                            int64_t n_rows,
                                                            const int64_t* __restrict__ dst_off,
                                                            T* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * 4 + wave_id();
  if (i >= n_rows) return;
  const int64_t r = rows ? rows[i] : i;
  const int64_t* o2 = off.at(r);
  const int64_t a = o2[0], n = o2[1] - a, o = dst_off[i];
  const T* s = r < src.n_a ? src.a : src.b;  // offsets are relative to the row's own source
  for (int64_t j = lane_id(); j < n; j += 64) dst[o + j] = s[a + j];
}

template <typename T>
__global__ void __launch_bounds__(256) take_kernel(Src2<T> src, const int64_t* __restrict__ rows,
                                                   int64_t n_rows, T* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n_rows) dst[i] = *src.at(rows ? rows[i] : i);
}

// Segmented index expansion: segment k covers outputs [seg_off[k], seg_off[k+1]); its element t
// is v = start + t * stride, written as v (mode 1) or src[v] (mode 0). One thread per output;
// the segment is found by binary search over the (L2-resident) segment offsets.
__global__ void __launch_bounds__(256) expand_segments_kernel(const int64_t* __restrict__ src,
                                                              const int64_t* __restrict__ seg,
                                                              const int64_t* __restrict__ seg_off,
                                                              int64_t n_seg, int64_t total,
                                                              int64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  int64_t lo = 0, hi = n_seg;  // seg_off[lo] <= i < seg_off[hi]
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (seg_off[mid] <= i) lo = mid;
    else hi = mid;
  }
  const int64_t v = seg[3 * lo] + (i - seg_off[lo]) * seg[3 * lo + 1];
  out[i] = seg[3 * lo + 2] ? v : src[v];
}

// Per-row metadata of the exchange: {len(A) + len(B), len(A), is_random_next, masks} as int32[4]
__global__ void __launch_bounds__(256) pairs_meta_pack_kernel(
    const int64_t* __restrict__ tok_off, const int32_t* __restrict__ len_a,
    const uint8_t* __restrict__ is_rn, const int64_t* __restrict__ pos_off,
    const int64_t* __restrict__ rows, int64_t n, int4* __restrict__ meta) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t r = rows ? rows[i] : i;
  meta[i] = make_int4((int32_t)(tok_off[r + 1] - tok_off[r]), len_a[r], (int32_t)is_rn[r],
                      pos_off ? (int32_t)(pos_off[r + 1] - pos_off[r]) : 0);
}

__global__ void __launch_bounds__(256) pairs_meta_unpack_kernel(
    const int4* __restrict__ meta, int64_t n, int64_t* __restrict__ ntok,
    int32_t* __restrict__ len_a, uint8_t* __restrict__ is_rn, int64_t* __restrict__ nmask) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int4 m = meta[i];
  ntok[i] = m.x;
  len_a[i] = m.y;
  is_rn[i] = (uint8_t)m.z;
  if (nmask) nmask[i] = m.w;
}

}  // namespace
}  // namespace lddl

using namespace lddl;

template <typename T>
static void launch_gather(const void* a, const int64_t* oa, int64_t n_a, const void* b,
                          const int64_t* ob, const int64_t* rows, int64_t n, const int64_t* dst_off,
                          void* dst, hipStream_t st) {
  hipLaunchKernelGGL(gather_ragged_kernel<T>, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st,
                     Src2<T>{(const T*)a, (const T*)b, n_a}, Src2<int64_t>{oa, ob, n_a}, rows, n,
                     dst_off, (T*)dst);
}

extern "C" int lddl_gather_ragged(void* stream, const void* d_src_a, const int64_t* d_off_a,
                                  int64_t n_a, const void* d_src_b, const int64_t* d_off_b,
                                  int32_t elem_bytes, const int64_t* d_rows, int64_t n_rows,
                                  const int64_t* d_dst_off, void* d_dst) {
  if (n_rows < 0 || n_a < 0) LDDL_FAIL(-1, "bad size");
  if (n_rows == 0) return 0;
  if (!d_rows && n_rows > n_a) LDDL_FAIL(-1, "n_rows > n_a without a row index");
  hipStream_t st = as_stream(stream);
  switch (elem_bytes) {
    case 1: launch_gather<uint8_t>(d_src_a, d_off_a, n_a, d_src_b, d_off_b, d_rows, n_rows, d_dst_off, d_dst, st); break;
    case 2: launch_gather<uint16_t>(d_src_a, d_off_a, n_a, d_src_b, d_off_b, d_rows, n_rows, d_dst_off, d_dst, st); break;
    case 4: launch_gather<uint32_t>(d_src_a, d_off_a, n_a, d_src_b, d_off_b, d_rows, n_rows, d_dst_off, d_dst, st); break;
    case 8: launch_gather<uint64_t>(d_src_a, d_off_a, n_a, d_src_b, d_off_b, d_rows, n_rows, d_dst_off, d_dst, st); break;
    default: LDDL_FAIL(-1, "elem_bytes %d unsupported", elem_bytes);
  }
  LDDL_HIP(hipGetLastError());
  return 0;
}

template <typename T>
static void launch_take(const void* a, int64_t n_a, const void* b, const int64_t* rows, int64_t n,
                        void* dst, hipStream_t st) {
  hipLaunchKernelGGL(take_kernel<T>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     Src2<T>{(const T*)a, (const T*)b, n_a}, rows, n, (T*)dst);
}

extern "C" int lddl_take(void* stream, const void* d_a, int64_t n_a, const void* d_b,
                         int32_t elem_bytes, const int64_t* d_rows, int64_t n_rows, void* d_dst) {
  if (n_rows < 0 || n_a < 0) LDDL_FAIL(-1, "bad size");
  if (n_rows == 0) return 0;
  if (!d_rows && n_rows > n_a) LDDL_FAIL(-1, "n_rows > n_a without a row index");
  hipStream_t st = as_stream(stream);
  switch (elem_bytes) {
    case 1: launch_take<uint8_t>(d_a, n_a, d_b, d_rows, n_rows, d_dst, st); break;
    case 2: launch_take<uint16_t>(d_a, n_a, d_b, d_rows, n_rows, d_dst, st); break;
    case 4: launch_take<uint32_t>(d_a, n_a, d_b, d_rows, n_rows, d_dst, st); break;
    case 8: launch_take<uint64_t>(d_a, n_a, d_b, d_rows, n_rows, d_dst, st); break;
    default: LDDL_FAIL(-1, "elem_bytes %d unsupported", elem_bytes);
  }
  LDDL_HIP(hipGetLastError());
  return 0;
}

extern "C" int lddl_expand_segments(void* stream, const int64_t* d_src, const int64_t* d_seg,
                                    const int64_t* d_seg_off, int64_t n_seg, int64_t total,
                                    int64_t* d_out) {
  if (n_seg < 0 || total < 0) LDDL_FAIL(-1, "bad size");
  if (total == 0) return 0;
  if (n_seg == 0) LDDL_FAIL(-1, "no segments for %lld outputs", (long long)total);
  hipLaunchKernelGGL(expand_segments_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     as_stream(stream), d_src, d_seg, d_seg_off, n_seg, total, d_out);
  LDDL_HIP(hipGetLastError());
  return 0;
}

namespace lddl {
namespace {
struct RowSize {
  Src2<int64_t> off;
  const int64_t* rows;
  __device__ int64_t operator()(int64_t i) const {
    const int64_t* o = off.at(rows ? rows[i] : i);
    return o[1] - o[0];
  }
};
}  // namespace
}  // namespace lddl

extern "C" int lddl_ragged_offsets(lddl_ctx* c, void* stream, const int64_t* d_off_a, int64_t n_a,
                                   const int64_t* d_off_b, const int64_t* d_rows, int64_t n_rows,
                                   int64_t* d_out) {
  if (!c) LDDL_FAIL(-1, "null ctx");
  if (n_rows < 0 || n_a < 0) LDDL_FAIL(-1, "bad size");
  if (!d_rows && n_rows > n_a) LDDL_FAIL(-1, "n_rows > n_a without a row index");
  hipStream_t st = as_stream(stream);
  ArenaTmp scratch(&c->arena, st);
  LDDL_HIP(scratch.take(sizeof(int64_t) * scan_scratch_elems(n_rows)));
  LDDL_HIP(scan_exclusive(RowSize{Src2<int64_t>{d_off_a, d_off_b, n_a}, d_rows}, n_rows, d_out,
                          scratch.as<int64_t>(), st));
  return 0;
}

extern "C" int lddl_pairs_meta_pack(void* stream, const int64_t* d_tok_off, const int32_t* d_len_a,
                                    const uint8_t* d_is_rn, const int64_t* d_pos_off,
                                    const int64_t* d_rows, int64_t n, int32_t* d_meta) {
  if (n < 0) LDDL_FAIL(-1, "bad size");
  if (n == 0) return 0;
  hipLaunchKernelGGL(pairs_meta_pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     as_stream(stream), d_tok_off, d_len_a, d_is_rn, d_pos_off, d_rows, n,
                     reinterpret_cast<int4*>(d_meta));
  LDDL_HIP(hipGetLastError());
  return 0;
}

extern "C" int lddl_pairs_meta_unpack(void* stream, const int32_t* d_meta, int64_t n,
                                      int64_t* d_ntok, int32_t* d_len_a, uint8_t* d_is_rn,
                                      int64_t* d_nmask) {
  if (n < 0) LDDL_FAIL(-1, "bad size");
  if (n == 0) return 0;
  hipLaunchKernelGGL(pairs_meta_unpack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     as_stream(stream), reinterpret_cast<const int4*>(d_meta), n, d_ntok, d_len_a,
                     d_is_rn, d_nmask);
  LDDL_HIP(hipGetLastError());
  return 0;
}

extern "C" int lddl_bin_partitions(lddl_ctx* c, void* stream, const int32_t* d_num_tokens,
                                   const int64_t* d_tok_off, int64_t n_rows,
                                   const int64_t* d_part_off, int64_t n_part, int32_t bin_size,
                                   int32_t nbins, int64_t* d_perm, int64_t* d_bin_id,
                                   int64_t* d_counts) {
  (void)c;
  if (bin_size < 1 || nbins < 1) LDDL_FAIL(-1, "bin_size and nbins must be >= 1");
  if (nbins > kMaxBinsLds) LDDL_FAIL(-1, "nbins %d > %d unsupported", nbins, kMaxBinsLds);
  if (n_part < 0 || n_rows < 0) LDDL_FAIL(-1, "bad sizes");
  if (!d_num_tokens && !d_tok_off && n_rows) LDDL_FAIL(-1, "need num_tokens or tok_off");
  if (n_part == 0) return 0;
  int nbits = 0;
  while ((1 << nbits) < nbins) ++nbits;
  hipLaunchKernelGGL(bin_partitions_kernel, dim3((unsigned)n_part), dim3(kBinThreads), 0,
                     as_stream(stream), NumTok{d_num_tokens, d_tok_off}, d_part_off, bin_size,
                     nbins, nbits, d_perm, d_bin_id, d_counts);
  LDDL_HIP(hipGetLastError());
  return 0;
}

extern "C" int lddl_bin_stable(lddl_ctx* c, void* stream, const int32_t* d_num_tokens,
                               const int64_t* d_tok_off, int64_t n_rows, int32_t bin_size,
                               int32_t nbins, int64_t* d_perm, int64_t* d_bin_id, int64_t* d_counts) {
  if (!c) LDDL_FAIL(-1, "null ctx");
  if (bin_size < 1 || nbins < 1) LDDL_FAIL(-1, "bin_size and nbins must be >= 1");
  if (nbins > kMaxBinsLds) LDDL_FAIL(-1, "nbins %d > %d unsupported", nbins, kMaxBinsLds);
  if (n_rows < 0) LDDL_FAIL(-1, "bad sizes");
  if (!d_num_tokens && !d_tok_off && n_rows) LDDL_FAIL(-1, "need num_tokens or tok_off");
  hipStream_t st = as_stream(stream);
  if (n_rows == 0) {
    LDDL_HIP(hipMemsetAsync(d_counts, 0, sizeof(int64_t) * nbins, st));
    return 0;
  }
  const NumTok nt{d_num_tokens, d_tok_off};
  int nbits = 0;
  while ((1 << nbits) < nbins) ++nbits;
  const int64_t n_tiles = (n_rows + kBinTile - 1) / kBinTile;
  const int64_t m = n_tiles * nbins;
  ArenaTmp tcb(&c->arena, st), scb(&c->arena, st);
  LDDL_HIP(tcb.take(sizeof(int64_t) * (2 * m + 1)));
  LDDL_HIP(scb.take(sizeof(int64_t) * scan_scratch_elems(m)));
  int64_t* tc = tcb.as<int64_t>();
  int64_t* base = tc + m;
  hipLaunchKernelGGL(bin_tile_hist_kernel, dim3((unsigned)n_tiles), dim3(64), 0, st, nt,
                     n_rows, bin_size, nbins, n_tiles, tc);
  struct In {
    const int64_t* v;
    __device__ int64_t operator()(int64_t i) const { return v[i]; }
  };
  LDDL_HIP(scan_exclusive(In{tc}, m, base, scb.as<int64_t>(), st));
  hipLaunchKernelGGL(bin_tile_scatter_kernel, dim3((unsigned)n_tiles), dim3(64), 0, st,
                     nt, n_rows, bin_size, nbins, nbits, n_tiles, base, d_perm, d_bin_id);
  hipLaunchKernelGGL(bin_totals_kernel, dim3((unsigned)((nbins + 255) / 256)), dim3(256), 0, st,
                     base, n_tiles, nbins, d_counts);
  LDDL_HIP(hipGetLastError());
  return 0;
}

static RenderArgs make_render(const lddl_ctx* c, const void* d_tokens, const int64_t* d_tok_off,
                              const int32_t* d_len_a, const uint16_t* d_pos, const void* d_lab,
                              const int64_t* d_pos_off, const int64_t* d_rows, int64_t n_rows) {
  return RenderArgs{c->d_render, c->d_render_off, d_tokens, d_tok_off, d_len_a, d_pos, d_lab,
                    d_pos_off, d_rows, n_rows, c->id_bytes()};
}

extern "C" int lddl_render_lengths(lddl_ctx* c, void* stream, const void* d_tokens,
                                   const int64_t* d_tok_off, const int32_t* d_len_a,
                                   const void* d_lab, const int64_t* d_pos_off,
                                   const int64_t* d_rows, int64_t n_rows, int64_t* d_a_len,
                                   int64_t* d_b_len, int64_t* d_l_len, int64_t* d_npy_len,
                                   const uint8_t* d_is_rn, uint16_t* d_num_tokens_out,
                                   uint8_t* d_is_rn_out) {
  if (!c) LDDL_FAIL(-1, "null ctx");
  if (n_rows <= 0) return 0;
  if (d_is_rn_out && !d_is_rn) LDDL_FAIL(-1, "is_random_next output without input");
  const RenderArgs R = make_render(c, d_tokens, d_tok_off, d_len_a, nullptr, d_lab, d_pos_off,
                                   d_rows, n_rows);
  hipLaunchKernelGGL(render_lengths_kernel, dim3((unsigned)((n_rows + 3) / 4)), dim3(256), 0,
                     as_stream(stream), R, d_a_len, d_b_len, d_l_len, d_npy_len, d_is_rn,
                     d_num_tokens_out, d_is_rn_out);
  LDDL_HIP(hipGetLastError());
  return 0;
}

extern "C" int lddl_render_write(lddl_ctx* c, void* stream, const void* d_tokens,
                                 const int64_t* d_tok_off, const int32_t* d_len_a,
                                 const uint16_t* d_pos, const void* d_lab,
                                 const int64_t* d_pos_off, const int64_t* d_rows, int64_t n_rows,
                                 const int64_t* d_a_off, const int64_t* d_b_off,
                                 const int64_t* d_l_off, const int64_t* d_npy_off,
                                 uint8_t* d_a_bytes, uint8_t* d_b_bytes, uint8_t* d_l_bytes,
                                 uint8_t* d_npy_bytes) {
  if (!c) LDDL_FAIL(-1, "null ctx");
  if (n_rows <= 0) return 0;
  const RenderArgs R = make_render(c, d_tokens, d_tok_off, d_len_a, d_pos, d_lab, d_pos_off, d_rows,
                                   n_rows);
  hipLaunchKernelGGL(render_write_kernel, dim3((unsigned)((n_rows + 3) / 4)), dim3(256), 0,
                     as_stream(stream), R, d_a_off, d_b_off, d_l_off, d_npy_off, d_a_bytes,
                     d_b_bytes, d_l_bytes, d_npy_bytes);
  LDDL_HIP(hipGetLastError());
  return 0;
}

extern "C" int lddl_scan_i64(lddl_ctx* c, void* stream, const int64_t* d_in, int64_t n,
                             int64_t* d_out) {
  if (!c) LDDL_FAIL(-1, "null ctx");
  if (n < 0) LDDL_FAIL(-1, "bad size");
  hipStream_t st = as_stream(stream);
  ArenaTmp scratch(&c->arena, st);
  LDDL_HIP(scratch.take(sizeof(int64_t) * scan_scratch_elems(n)));
  struct In {
    const int64_t* v;
    __device__ int64_t operator()(int64_t i) const { return v[i]; }
  };
  LDDL_HIP(scan_exclusive(In{d_in}, n, d_out, scratch.as<int64_t>(), st));
  return 0;
}
