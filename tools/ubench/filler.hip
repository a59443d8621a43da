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

__global__ void __launch_bounds__(256) salu_filler(int iters, int* sink) {
  int s0 = threadIdx.x >> 6, s1 = s0 + 1, s2 = s0 + 2, s3 = s0 + 3, s4 = s0 + 4, s5 = s0 + 5, s6 = s0 + 6, s7 = s0 + 7;
  s0 = __builtin_amdgcn_readfirstlane(s0); s1 = __builtin_amdgcn_readfirstlane(s1);
  s2 = __builtin_amdgcn_readfirstlane(s2); s3 = __builtin_amdgcn_readfirstlane(s3);
  s4 = __builtin_amdgcn_readfirstlane(s4); s5 = __builtin_amdgcn_readfirstlane(s5);
  s6 = __builtin_amdgcn_readfirstlane(s6); s7 = __builtin_amdgcn_readfirstlane(s7);
  for (int it = 0; it < iters; ++it) {
    asm volatile(
        "s_add_u32 %0, %0, 1\n s_add_u32 %1, %1, 1\n s_add_u32 %2, %2, 1\n s_add_u32 %3, %3, 1\n"
        "s_add_u32 %4, %4, 1\n s_add_u32 %5, %5, 1\n s_add_u32 %6, %6, 1\n s_add_u32 %7, %7, 1\n"
        "s_add_u32 %0, %0, 1\n s_add_u32 %1, %1, 1\n s_add_u32 %2, %2, 1\n s_add_u32 %3, %3, 1\n"
        "s_add_u32 %4, %4, 1\n s_add_u32 %5, %5, 1\n s_add_u32 %6, %6, 1\n s_add_u32 %7, %7, 1\n"
        "s_add_u32 %0, %0, 1\n s_add_u32 %1, %1, 1\n s_add_u32 %2, %2, 1\n s_add_u32 %3, %3, 1\n"
        "s_add_u32 %4, %4, 1\n s_add_u32 %5, %5, 1\n s_add_u32 %6, %6, 1\n s_add_u32 %7, %7, 1\n"
        "s_add_u32 %0, %0, 1\n s_add_u32 %1, %1, 1\n s_add_u32 %2, %2, 1\n s_add_u32 %3, %3, 1\n"
        "s_add_u32 %4, %4, 1\n s_add_u32 %5, %5, 1\n s_add_u32 %6, %6, 1\n s_add_u32 %7, %7, 1\n"
        : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7) :: "scc");
  }
  const int r = s0 + s1 + s2 + s3 + s4 + s5 + s6 + s7;
  if (r == 0x7fffffff && threadIdx.x == 0) sink[0] = r;
}

extern "C" int ubench_salu_filler(void* stream, int blocks, int iters, int* sink) {
  hipLaunchKernelGGL(salu_filler, dim3(blocks), dim3(256), 0, (hipStream_t)stream, iters, sink);
  return (int)hipGetLastError();
}

extern "C" int ubench_valu_filler(void* stream, int blocks, int iters, int* sink) {
  hipLaunchKernelGGL(valu_filler, dim3(blocks), dim3(256), 0, (hipStream_t)stream, iters, sink);
  return (int)hipGetLastError();
}
