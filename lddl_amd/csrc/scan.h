// Device-wide exclusive prefix sum over int64 values produced by a functor f(i), i in [0, n).
// Three launches: per-block reduce -> single-block scan of block sums -> per-block scan + write.
// out[0..n] gets the exclusive scan with out[n] = total.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "device.h"

namespace lddl {

constexpr int kScanThreads = 256;
constexpr int kScanItems = 8;
constexpr int64_t kScanTile = kScanThreads * kScanItems;

__device__ inline int64_t block_excl_scan(int64_t v, int64_t* total) {
  __shared__ int64_t wsum[kScanThreads / 64];
  const int w = threadIdx.x >> 6;
  const int64_t incl = wave_incl_scan(v);
  if (lane_id() == 63) wsum[w] = incl;
  __syncthreads();
  int64_t off = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < kScanThreads / 64; ++k) {
    if (k < w) off += wsum[k];
    tot += wsum[k];
  }
  __syncthreads();
  *total = tot;
  return off + incl - v;
}

template <typename F>
__global__ void __launch_bounds__(kScanThreads) scan_reduce_kernel(F f, int64_t n, int64_t* sums) {
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  int64_t v = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k)
    if (base + k < n) v += f(base + k);
  int64_t tot;
  block_excl_scan(v, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// exclusive scan of sums[0..nb) in place, sums[nb] = total (one workgroup)
__global__ void __launch_bounds__(kScanThreads) scan_sums_kernel(int64_t* sums, int64_t nb);

template <typename F>
__global__ void __launch_bounds__(kScanThreads) scan_write_kernel(F f, int64_t n, const int64_t* sums,
                                                                 int64_t* out) {
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  int64_t vals[kScanItems];
  int64_t v = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    vals[k] = base + k < n ? f(base + k) : 0;
    v += vals[k];
  }
  int64_t tot;
  int64_t off = block_excl_scan(v, &tot) + sums[blockIdx.x];
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    if (base + k < n) out[base + k] = off;
    off += vals[k];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == kScanThreads - 1) out[n] = sums[gridDim.x];
}

// Scratch for scan_exclusive: (n / kScanTile + 2) int64.
inline int64_t scan_scratch_elems(int64_t n) { return (n + kScanTile - 1) / kScanTile + 2; }

template <typename F>
hipError_t scan_exclusive(F f, int64_t n, int64_t* out, int64_t* scratch, hipStream_t st) {
  const int64_t nb = n > 0 ? (n + kScanTile - 1) / kScanTile : 1;
  hipLaunchKernelGGL(scan_reduce_kernel<F>, dim3((unsigned)nb), dim3(kScanThreads), 0, st, f, n,
                     scratch);
  hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(kScanThreads), 0, st, scratch, nb);
  hipLaunchKernelGGL(scan_write_kernel<F>, dim3((unsigned)nb), dim3(kScanThreads), 0, st, f, n,
                     scratch, out);
  return hipGetLastError();
}

// Two exclusive scans in one set of passes over a functor returning both values (Sum2): each
// input element is read once; out_a / out_b as scan_exclusive's out. Scratch: twice
// scan_scratch_elems(n).
struct Sum2 {
  int64_t a, b;
};

template <typename F>
__global__ void __launch_bounds__(kScanThreads) scan_reduce2_kernel(F f, int64_t n, int64_t* sa, int64_t* sb) {
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  int64_t va = 0, vb = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k)
    if (base + k < n) {
      const Sum2 s = f(base + k);
      va += s.a;
      vb += s.b;
    }
  int64_t ta, tb;
  block_excl_scan(va, &ta);
  block_excl_scan(vb, &tb);
  if (threadIdx.x == 0) {
    sa[blockIdx.x] = ta;
    sb[blockIdx.x] = tb;
  }
}

// sa (block 0) and sb (block 1) as scan_sums_kernel
__global__ void __launch_bounds__(kScanThreads) scan_sums2_kernel(int64_t* sa, int64_t* sb, int64_t nb);

template <typename F>
__global__ void __launch_bounds__(kScanThreads) scan_write2_kernel(F f, int64_t n, const int64_t* sa,
                                                                  const int64_t* sb, int64_t* oa,
                                                                  int64_t* ob) {
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  Sum2 vals[kScanItems];
  int64_t va = 0, vb = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    vals[k] = base + k < n ? f(base + k) : Sum2{0, 0};
    va += vals[k].a;
    vb += vals[k].b;
  }
  int64_t ta, tb;
  int64_t offa = block_excl_scan(va, &ta) + sa[blockIdx.x];
  int64_t offb = block_excl_scan(vb, &tb) + sb[blockIdx.x];
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    if (base + k < n) {
      oa[base + k] = offa;
      ob[base + k] = offb;
    }
    offa += vals[k].a;
    offb += vals[k].b;
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == kScanThreads - 1) {
    oa[n] = sa[gridDim.x];
    ob[n] = sb[gridDim.x];
  }
}

template <typename F>
hipError_t scan_exclusive2(F f, int64_t n, int64_t* out_a, int64_t* out_b, int64_t* scratch,
                           hipStream_t st) {
  const int64_t nb = n > 0 ? (n + kScanTile - 1) / kScanTile : 1;
  int64_t* sb = scratch + scan_scratch_elems(n);
  hipLaunchKernelGGL(scan_reduce2_kernel<F>, dim3((unsigned)nb), dim3(kScanThreads), 0, st, f, n,
                     scratch, sb);
  hipLaunchKernelGGL(scan_sums2_kernel, dim3(2), dim3(kScanThreads), 0, st, scratch, sb, nb);
  hipLaunchKernelGGL(scan_write2_kernel<F>, dim3((unsigned)nb), dim3(kScanThreads), 0, st, f, n,
                     scratch, sb, out_a, out_b);
  return hipGetLastError();
}

}  // namespace lddl
