// VALU-only filler kernel for the co-residency experiment (tools/corun_planner.py; diagnostic,
// not product): `blocks` workgroups of 256 threads (one wave per SIMD when blocks = CUs), each
// wave running `iters` x 32 independent v_add_u32 (8 chains). Loaded with ctypes; launched on the
// caller's stream.
#include <hip/hip_runtime.h>

__global__ void __launch_bounds__(256) valu_filler(int iters, int* sink) {
  int v0 = threadIdx.x, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4, v5 = v0 + 5, v6 = v0 + 6, v7 = v0 + 7;
  for (int it = 0; it < iters; ++it) {
    asm volatile(
        "v_add_u32 %0, %0, 1\n v_add_u32 %1, %1, 1\n v_add_u32 %2, %2, 1\n v_add_u32 %3, %3, 1\n"
        "v_add_u32 %4, %4, 1\n v_add_u32 %5, %5, 1\n v_add_u32 %6, %6, 1\n v_add_u32 %7, %7, 1\n"
        "v_add_u32 %0, %0, 1\n v_add_u32 %1, %1, 1\n v_add_u32 %2, %2, 1\n v_add_u32 %3, %3, 1\n"
        "v_add_u32 %4, %4, 1\n v_add_u32 %5, %5, 1\n v_add_u32 %6, %6, 1\n v_add_u32 %7, %7, 1\n"
        "v_add_u32 %0, %0, 1\n v_add_u32 %1, %1, 1\n v_add_u32 %2, %2, 1\n v_add_u32 %3, %3, 1\n"
        "v_add_u32 %4, %4, 1\n v_add_u32 %5, %5, 1\n v_add_u32 %6, %6, 1\n v_add_u32 %7, %7, 1\n"
        "v_add_u32 %0, %0, 1\n v_add_u32 %1, %1, 1\n v_add_u32 %2, %2, 1\n v_add_u32 %3, %3, 1\n"
        "v_add_u32 %4, %4, 1\n v_add_u32 %5, %5, 1\n v_add_u32 %6, %6, 1\n v_add_u32 %7, %7, 1\n"
        : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7));
  }
  const int r = v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7;
  if (r == 0x7fffffff) sink[0] = r;
}

extern "C" int ubench_valu_filler(void* stream, int blocks, int iters, int* sink) {
  hipLaunchKernelGGL(valu_filler, dim3(blocks), dim3(256), 0, (hipStream_t)stream, iters, sink);
  return (int)hipGetLastError();
}
