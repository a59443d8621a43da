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

__global__ void __launch_bounds__(kBinThreads) bin_partitions_kernel(
    const int32_t* __restrict__ num_tokens, const int64_t* __restrict__ part_off, int32_t bin_size,
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

__global__ void __launch_bounds__(64) bin_tile_hist_kernel(const int32_t* __restrict__ num_tokens,
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
    const int32_t* __restrict__ num_tokens, int64_t n, int32_t bin_size, int32_t nbins,
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
      bin_id[dst] = b;
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
  const int32_t* tokens;
  const int64_t* tok_off;
  const int32_t* len_a;
  const uint16_t* pos;
  const int32_t* lab;
  const int64_t* pos_off;
  const int64_t* rows;  // output row -> pair (NULL: identity)
  int64_t n_rows;
};

__device__ inline int32_t tok_len(const RenderArgs& R, int32_t id) {
  return (int32_t)(R.roff[id + 1] - R.roff[id]);
}

// total bytes of ' '.join(strings of ids[0..n))
__device__ int64_t joined_len(const RenderArgs& R, const int32_t* ids, int64_t n) {
  int64_t acc = 0;
  for (int64_t c0 = 0; c0 < n; c0 += 64) {
    const int64_t j = c0 + lane_id();
    acc += j < n ? tok_len(R, ids[j]) : 0;
  }
  return wave_sum(acc) + (n > 0 ? n - 1 : 0);
}

__device__ void joined_write(const RenderArgs& R, const int32_t* ids, int64_t n, uint8_t* out) {
  int64_t base = 0;
  for (int64_t c0 = 0; c0 < n; c0 += 64) {
    const int64_t j = c0 + lane_id();
    const int32_t id = j < n ? ids[j] : 0;
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
                                                             int64_t* n_pos) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R.n_rows) return;
  const int64_t q = R.rows ? R.rows[row] : row;
  const int64_t t0 = R.tok_off[q], t1 = R.tok_off[q + 1];
  const int32_t na = R.len_a[q];
  const int64_t la = joined_len(R, R.tokens + t0, na);
  const int64_t lb = joined_len(R, R.tokens + t0 + na, t1 - t0 - na);
  int64_t ll = 0, np = 0;
  if (R.pos_off) {
    const int64_t p0 = R.pos_off[q], p1 = R.pos_off[q + 1];
    ll = joined_len(R, R.lab + p0, p1 - p0);
    np = p1 - p0;
  }
  if (lane_id() == 0) {
    a_len[row] = la;
    b_len[row] = lb;
    if (l_len) l_len[row] = ll;
    if (n_pos) n_pos[row] = 128 + 2 * np;
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
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R.n_rows) return;
  const int64_t q = R.rows ? R.rows[row] : row;
  const int64_t t0 = R.tok_off[q], t1 = R.tok_off[q + 1];
  const int32_t na = R.len_a[q];
  joined_write(R, R.tokens + t0, na, a_bytes + a_off[row]);
  joined_write(R, R.tokens + t0 + na, t1 - t0 - na, b_bytes + b_off[row]);
  if (R.pos_off) {
    const int64_t p0 = R.pos_off[q], p1 = R.pos_off[q + 1];
    if (l_bytes) joined_write(R, R.lab + p0, p1 - p0, l_bytes + l_off[row]);
    if (npy_bytes) put_npy(npy_bytes + npy_off[row], R.pos + p0, p1 - p0);
  }
}

// ---- ragged row gather (sample exchange packing) ---------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) gather_ragged_kernel(const T* __restrict__ src,
                                                            const int64_t* __restrict__ src_off,
                                                            const int64_t* __restrict__ rows,
                                                            int64_t n_rows,
                                                            const int64_t* __restrict__ dst_off,
                                                            T* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n_rows) return;
  const int64_t r = rows ? rows[i] : i;
  const int64_t a = src_off[r], n = src_off[r + 1] - a, o = dst_off[i];
  for (int64_t j = lane_id(); j < n; j += 64) dst[o + j] = src[a + j];
}

}  // namespace
}  // namespace lddl

using namespace lddl;

extern "C" int lddl_gather_ragged(void* stream, const void* d_src, const int64_t* d_src_off,
                                  int32_t elem_bytes, const int64_t* d_rows, int64_t n_rows,
                                  const int64_t* d_dst_off, void* d_dst) {
  if (n_rows < 0) LDDL_FAIL(-1, "bad size");
  if (n_rows == 0) return 0;
  const dim3 grid((unsigned)((n_rows + 3) / 4)), block(256);
  hipStream_t st = as_stream(stream);
  switch (elem_bytes) {
    case 1:
      hipLaunchKernelGGL(gather_ragged_kernel<uint8_t>, grid, block, 0, st,
                         (const uint8_t*)d_src, d_src_off, d_rows, n_rows, d_dst_off, (uint8_t*)d_dst);
      break;
    case 2:
      hipLaunchKernelGGL(gather_ragged_kernel<uint16_t>, grid, block, 0, st,
                         (const uint16_t*)d_src, d_src_off, d_rows, n_rows, d_dst_off, (uint16_t*)d_dst);
      break;
    case 4:
      hipLaunchKernelGGL(gather_ragged_kernel<uint32_t>, grid, block, 0, st,
                         (const uint32_t*)d_src, d_src_off, d_rows, n_rows, d_dst_off, (uint32_t*)d_dst);
      break;
    case 8:
      hipLaunchKernelGGL(gather_ragged_kernel<uint64_t>, grid, block, 0, st,
                         (const uint64_t*)d_src, d_src_off, d_rows, n_rows, d_dst_off, (uint64_t*)d_dst);
      break;
    default:
      LDDL_FAIL(-1, "elem_bytes %d unsupported", elem_bytes);
  }
  LDDL_HIP(hipGetLastError());
  return 0;
}

extern "C" int lddl_bin_partitions(lddl_ctx* c, void* stream, const int32_t* d_num_tokens,
                                   int64_t n_rows, const int64_t* d_part_off, int64_t n_part,
                                   int32_t bin_size, int32_t nbins, int64_t* d_perm,
                                   int64_t* d_bin_id, int64_t* d_counts) {
  (void)c;
  if (bin_size < 1 || nbins < 1) LDDL_FAIL(-1, "bin_size and nbins must be >= 1");
  if (nbins > kMaxBinsLds) LDDL_FAIL(-1, "nbins %d > %d unsupported", nbins, kMaxBinsLds);
  if (n_part < 0 || n_rows < 0) LDDL_FAIL(-1, "bad sizes");
  if (n_part == 0) return 0;
  int nbits = 0;
  while ((1 << nbits) < nbins) ++nbits;
  hipLaunchKernelGGL(bin_partitions_kernel, dim3((unsigned)n_part), dim3(kBinThreads), 0,
                     as_stream(stream), d_num_tokens, d_part_off, bin_size, nbins, nbits, d_perm,
                     d_bin_id, d_counts);
  LDDL_HIP(hipGetLastError());
  return 0;
}

extern "C" int lddl_bin_stable(lddl_ctx* c, void* stream, const int32_t* d_num_tokens,
                               int64_t n_rows, int32_t bin_size, int32_t nbins, int64_t* d_perm,
                               int64_t* d_bin_id, int64_t* d_counts) {
  (void)c;
  if (bin_size < 1 || nbins < 1) LDDL_FAIL(-1, "bin_size and nbins must be >= 1");
  if (nbins > kMaxBinsLds) LDDL_FAIL(-1, "nbins %d > %d unsupported", nbins, kMaxBinsLds);
  if (n_rows < 0) LDDL_FAIL(-1, "bad sizes");
  hipStream_t st = as_stream(stream);
  if (n_rows == 0) {
    LDDL_HIP(hipMemsetAsync(d_counts, 0, sizeof(int64_t) * nbins, st));
    return 0;
  }
  int nbits = 0;
  while ((1 << nbits) < nbins) ++nbits;
  const int64_t n_tiles = (n_rows + kBinTile - 1) / kBinTile;
  const int64_t m = n_tiles * nbins;
  int64_t *tc, *scratch;
  LDDL_HIP(hipMallocAsync((void**)&tc, sizeof(int64_t) * (2 * m + 1), st));
  LDDL_HIP(hipMallocAsync((void**)&scratch, sizeof(int64_t) * scan_scratch_elems(m), st));
  int64_t* base = tc + m;
  hipLaunchKernelGGL(bin_tile_hist_kernel, dim3((unsigned)n_tiles), dim3(64), 0, st, d_num_tokens,
                     n_rows, bin_size, nbins, n_tiles, tc);
  struct In {
    const int64_t* v;
    __device__ int64_t operator()(int64_t i) const { return v[i]; }
  };
  const hipError_t e = scan_exclusive(In{tc}, m, base, scratch, st);
  hipLaunchKernelGGL(bin_tile_scatter_kernel, dim3((unsigned)n_tiles), dim3(64), 0, st,
                     d_num_tokens, n_rows, bin_size, nbins, nbits, n_tiles, base, d_perm, d_bin_id);
  hipLaunchKernelGGL(bin_totals_kernel, dim3((unsigned)((nbins + 255) / 256)), dim3(256), 0, st,
                     base, n_tiles, nbins, d_counts);
  LDDL_HIP(hipFreeAsync(scratch, st));
  LDDL_HIP(hipFreeAsync(tc, st));
  LDDL_HIP(e);
  LDDL_HIP(hipGetLastError());
  return 0;
}

static RenderArgs make_render(const lddl_ctx* c, const int32_t* d_tokens, const int64_t* d_tok_off,
                              const int32_t* d_len_a, const uint16_t* d_pos, const int32_t* d_lab,
                              const int64_t* d_pos_off, const int64_t* d_rows, int64_t n_rows) {
  return RenderArgs{c->d_render, c->d_render_off, d_tokens, d_tok_off, d_len_a, d_pos, d_lab,
                    d_pos_off, d_rows, n_rows};
}

extern "C" int lddl_render_lengths(lddl_ctx* c, void* stream, const int32_t* d_tokens,
                                   const int64_t* d_tok_off, const int32_t* d_len_a,
                                   const int32_t* d_lab, const int64_t* d_pos_off,
                                   const int64_t* d_rows, int64_t n_rows, int64_t* d_a_len,
                                   int64_t* d_b_len, int64_t* d_l_len, int64_t* d_npy_len) {
  if (!c) LDDL_FAIL(-1, "null ctx");
  if (n_rows <= 0) return 0;
  const RenderArgs R = make_render(c, d_tokens, d_tok_off, d_len_a, nullptr, d_lab, d_pos_off,
                                   d_rows, n_rows);
  hipLaunchKernelGGL(render_lengths_kernel, dim3((unsigned)((n_rows + 3) / 4)), dim3(256), 0,
                     as_stream(stream), R, d_a_len, d_b_len, d_l_len, d_npy_len);
  LDDL_HIP(hipGetLastError());
  return 0;
}

extern "C" int lddl_render_write(lddl_ctx* c, void* stream, const int32_t* d_tokens,
                                 const int64_t* d_tok_off, const int32_t* d_len_a,
                                 const uint16_t* d_pos, const int32_t* d_lab,
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

extern "C" int lddl_scan_i64(void* stream, const int64_t* d_in, int64_t n, int64_t* d_out) {
  if (n < 0) LDDL_FAIL(-1, "bad size");
  hipStream_t st = as_stream(stream);
  int64_t* scratch;
  LDDL_HIP(hipMallocAsync((void**)&scratch, sizeof(int64_t) * scan_scratch_elems(n), st));
  struct In {
    const int64_t* v;
    __device__ int64_t operator()(int64_t i) const { return v[i]; }
  };
  const hipError_t e = scan_exclusive(In{d_in}, n, d_out, scratch, st);
  LDDL_HIP(hipFreeAsync(scratch, st));
  LDDL_HIP(e);
  return 0;
}
