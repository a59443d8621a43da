#include "scan.h"

namespace lddl {

__device__ void scan_sums_block(int64_t* sums, int64_t nb) {
  int64_t carry = 0;
  for (int64_t b0 = 0; b0 < nb; b0 += kScanThreads) {
    const int64_t i = b0 + threadIdx.x;
    const int64_t v = i < nb ? sums[i] : 0;
    int64_t tot;
    const int64_t ex = block_excl_scan(v, &tot);
    if (i < nb) sums[i] = carry + ex;
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) sums[nb] = carry;
}

__global__ void __launch_bounds__(kScanThreads) scan_sums_kernel(int64_t* sums, int64_t nb) {
  scan_sums_block(sums, nb);
}

__global__ void __launch_bounds__(kScanThreads) scan_sums2_kernel(int64_t* sa, int64_t* sb, int64_t nb) {
  scan_sums_block(blockIdx.x ? sb : sa, nb);
}

}  // namespace lddl
