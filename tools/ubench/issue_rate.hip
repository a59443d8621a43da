// Issue-rate probe for gfx950 (diagnostic, not product): SALU vs VALU vs mixed instruction
// throughput per SIMD at 1, 2, 4 and 8 waves per SIMD, and 32-bit vs 24-bit integer multiplies. Each wave runs ITER x 32 independent
// adds (8 registers round robin); cycles from s_memtime (shader clock) per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <string>
#include <vector>

constexpr int ITER = 4096;

#define S8(op) op(0) op(1) op(2) op(3) op(4) op(5) op(6) op(7)
template <int MODE>
__global__ void probe(unsigned long long* cyc, int* sink) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  int s0 = threadIdx.x >> 6, s1 = s0 + 1, s2 = s0 + 2, s3 = s0 + 3, s4 = s0 + 4, s5 = s0 + 5, s6 = s0 + 6, s7 = s0 + 7;
  s0 = __builtin_amdgcn_readfirstlane(s0); s1 = __builtin_amdgcn_readfirstlane(s1);
  s2 = __builtin_amdgcn_readfirstlane(s2); s3 = __builtin_amdgcn_readfirstlane(s3);
  s4 = __builtin_amdgcn_readfirstlane(s4); s5 = __builtin_amdgcn_readfirstlane(s5);
  s6 = __builtin_amdgcn_readfirstlane(s6); s7 = __builtin_amdgcn_readfirstlane(s7);
  int v0 = threadIdx.x, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4, v5 = v0 + 5, v6 = v0 + 6, v7 = v0 + 7;
  for (int it = 0; it < ITER; ++it) {
    if (MODE == 0) {  // 32 SALU
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
    } else if (MODE == 1) {  // 32 VALU
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
    } else if (MODE == 3) {  // 32 v_mul_lo_u32 (8 independent chains)
      asm volatile(
          "v_mul_lo_u32 %0, %0, %8\n v_mul_lo_u32 %1, %1, %8\n v_mul_lo_u32 %2, %2, %8\n v_mul_lo_u32 %3, %3, %8\n"
          "v_mul_lo_u32 %4, %4, %8\n v_mul_lo_u32 %5, %5, %8\n v_mul_lo_u32 %6, %6, %8\n v_mul_lo_u32 %7, %7, %8\n"
          "v_mul_lo_u32 %0, %0, %8\n v_mul_lo_u32 %1, %1, %8\n v_mul_lo_u32 %2, %2, %8\n v_mul_lo_u32 %3, %3, %8\n"
          "v_mul_lo_u32 %4, %4, %8\n v_mul_lo_u32 %5, %5, %8\n v_mul_lo_u32 %6, %6, %8\n v_mul_lo_u32 %7, %7, %8\n"
          "v_mul_lo_u32 %0, %0, %8\n v_mul_lo_u32 %1, %1, %8\n v_mul_lo_u32 %2, %2, %8\n v_mul_lo_u32 %3, %3, %8\n"
          "v_mul_lo_u32 %4, %4, %8\n v_mul_lo_u32 %5, %5, %8\n v_mul_lo_u32 %6, %6, %8\n v_mul_lo_u32 %7, %7, %8\n"
          "v_mul_lo_u32 %0, %0, %8\n v_mul_lo_u32 %1, %1, %8\n v_mul_lo_u32 %2, %2, %8\n v_mul_lo_u32 %3, %3, %8\n"
          "v_mul_lo_u32 %4, %4, %8\n v_mul_lo_u32 %5, %5, %8\n v_mul_lo_u32 %6, %6, %8\n v_mul_lo_u32 %7, %7, %8\n"
          : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(s0 + 3));
    } else if (MODE == 4) {  // 32 v_mad_u32_u24 (8 independent chains)
      asm volatile(
          "v_mad_u32_u24 %0, %0, %8, %8\n v_mad_u32_u24 %1, %1, %8, %8\n v_mad_u32_u24 %2, %2, %8, %8\n v_mad_u32_u24 %3, %3, %8, %8\n"
          "v_mad_u32_u24 %4, %4, %8, %8\n v_mad_u32_u24 %5, %5, %8, %8\n v_mad_u32_u24 %6, %6, %8, %8\n v_mad_u32_u24 %7, %7, %8, %8\n"
          "v_mad_u32_u24 %0, %0, %8, %8\n v_mad_u32_u24 %1, %1, %8, %8\n v_mad_u32_u24 %2, %2, %8, %8\n v_mad_u32_u24 %3, %3, %8, %8\n"
          "v_mad_u32_u24 %4, %4, %8, %8\n v_mad_u32_u24 %5, %5, %8, %8\n v_mad_u32_u24 %6, %6, %8, %8\n v_mad_u32_u24 %7, %7, %8, %8\n"
          "v_mad_u32_u24 %0, %0, %8, %8\n v_mad_u32_u24 %1, %1, %8, %8\n v_mad_u32_u24 %2, %2, %8, %8\n v_mad_u32_u24 %3, %3, %8, %8\n"
          "v_mad_u32_u24 %4, %4, %8, %8\n v_mad_u32_u24 %5, %5, %8, %8\n v_mad_u32_u24 %6, %6, %8, %8\n v_mad_u32_u24 %7, %7, %8, %8\n"
          "v_mad_u32_u24 %0, %0, %8, %8\n v_mad_u32_u24 %1, %1, %8, %8\n v_mad_u32_u24 %2, %2, %8, %8\n v_mad_u32_u24 %3, %3, %8, %8\n"
          "v_mad_u32_u24 %4, %4, %8, %8\n v_mad_u32_u24 %5, %5, %8, %8\n v_mad_u32_u24 %6, %6, %8, %8\n v_mad_u32_u24 %7, %7, %8, %8\n"
          : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(s0 + 3));
    } else {  // 16 SALU + 16 VALU interleaved
      asm volatile(
          "s_add_u32 %0, %0, 1\n v_add_u32 %8, %8, 1\n s_add_u32 %1, %1, 1\n v_add_u32 %9, %9, 1\n"
          "s_add_u32 %2, %2, 1\n v_add_u32 %10, %10, 1\n s_add_u32 %3, %3, 1\n v_add_u32 %11, %11, 1\n"
          "s_add_u32 %4, %4, 1\n v_add_u32 %12, %12, 1\n s_add_u32 %5, %5, 1\n v_add_u32 %13, %13, 1\n"
          "s_add_u32 %6, %6, 1\n v_add_u32 %14, %14, 1\n s_add_u32 %7, %7, 1\n v_add_u32 %15, %15, 1\n"
          "s_add_u32 %0, %0, 1\n v_add_u32 %8, %8, 1\n s_add_u32 %1, %1, 1\n v_add_u32 %9, %9, 1\n"
          "s_add_u32 %2, %2, 1\n v_add_u32 %10, %10, 1\n s_add_u32 %3, %3, 1\n v_add_u32 %11, %11, 1\n"
          "s_add_u32 %4, %4, 1\n v_add_u32 %12, %12, 1\n s_add_u32 %5, %5, 1\n v_add_u32 %13, %13, 1\n"
          "s_add_u32 %6, %6, 1\n v_add_u32 %14, %14, 1\n s_add_u32 %7, %7, 1\n v_add_u32 %15, %15, 1\n"
          : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7),
            "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) :: "scc");
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const int w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if ((threadIdx.x & 63) == 0) cyc[w] = t1 - t0;
  const int r = s0 + s1 + s2 + s3 + s4 + s5 + s6 + s7 + v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7;
  if (r == 0x7fffffff) sink[0] = r;
}

// Co-residency: a SALU-only kernel and a VALU-only kernel on two streams at
// the same time, each with `wps` waves per SIMD, against each alone. If the CU's scalar unit and
// the SIMDs' vector pipes serve different waves in the same cycles, the pair takes ~max of the
// two alone; if issue is shared, ~their sum.
static void corun(int ncu, unsigned long long* cyc, unsigned long long* cyc2, int* sink) {
  hipStream_t s1, s2;
  hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  const int reps = 20;
  for (int wps : {1, 2, 4}) {
    const int threads = 256 * wps, blocks = ncu;
    auto run = [&](bool sa, bool va, float* t_s, float* t_v, float* t_all) {
      hipEvent_t a, b1, b2;
      hipEventCreate(&a);
      hipEventCreate(&b1);
      hipEventCreate(&b2);
      hipDeviceSynchronize();
      hipEventRecord(a, 0);
      hipDeviceSynchronize();
      for (int r = 0; r < reps; ++r) {
        if (sa) hipLaunchKernelGGL(probe<0>, dim3(blocks), dim3(threads), 0, s1, cyc, sink);
        if (va) hipLaunchKernelGGL(probe<1>, dim3(blocks), dim3(threads), 0, s2, cyc2, sink);
      }
      hipEventRecord(b1, s1);
      hipEventRecord(b2, s2);
      hipEventSynchronize(b1);
      hipEventSynchronize(b2);
      float x = 0, y = 0;
      hipEventElapsedTime(&x, a, b1);
      hipEventElapsedTime(&y, a, b2);
      if (t_s) *t_s = x;
      if (t_v) *t_v = y;
      if (t_all) *t_all = x > y ? x : y;
    };
    float ts = 0, tv = 0, cs = 0, cv = 0, call = 0;
    run(true, false, &ts, nullptr, nullptr);
    run(false, true, nullptr, &tv, nullptr);
    run(true, true, &cs, &cv, &call);
    printf("corun waves/SIMD %d+%d: SALU alone %.3f ms, VALU alone %.3f ms (sum %.3f, max %.3f); "
           "together: SALU stream %.3f ms, VALU stream %.3f ms, both done %.3f ms -> overlap %.0f%%\n",
           wps, wps, ts, tv, ts + tv, ts > tv ? ts : tv, cs, cv, call,
           100.0 * (ts + tv - call) / (ts < tv ? ts : tv));
  }
}

int main(int argc, char** argv) {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  unsigned long long* cyc;
  int* sink;
  hipMalloc(&cyc, sizeof(unsigned long long) * ncu * 32);
  hipMalloc(&sink, 4);
  if (argc > 1 && std::string(argv[1]) == "corun") {
    unsigned long long* cyc2;
    hipMalloc(&cyc2, sizeof(unsigned long long) * ncu * 32);
    corun(ncu, cyc, cyc2, sink);
    return 0;
  }
  const char* names[5] = {"salu32", "valu32", "mix16+16", "mul_lo32", "mad_u24"};
  for (int mode = 0; mode < 5; ++mode) {
    for (int wps : {1, 2, 4, 8}) {  // waves per SIMD: workgroups of 4 * wps waves, one per CU
      const int threads = 256 * wps > 1024 ? 1024 : 256 * wps;
      const int blocks = ncu * (256 * wps / threads);
      hipEvent_t a, b;
      hipEventCreate(&a);
      hipEventCreate(&b);
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(a);
        if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(blocks), dim3(threads), 0, 0, cyc, sink);
        if (mode == 1) hipLaunchKernelGGL(probe<1>, dim3(blocks), dim3(threads), 0, 0, cyc, sink);
        if (mode == 2) hipLaunchKernelGGL(probe<2>, dim3(blocks), dim3(threads), 0, 0, cyc, sink);
        if (mode == 3) hipLaunchKernelGGL(probe<3>, dim3(blocks), dim3(threads), 0, 0, cyc, sink);
        if (mode == 4) hipLaunchKernelGGL(probe<4>, dim3(blocks), dim3(threads), 0, 0, cyc, sink);
        hipEventRecord(b);
        hipEventSynchronize(b);
      }
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      const int nw = blocks * threads / 64;
      std::vector<unsigned long long> h(nw);
      hipMemcpy(h.data(), cyc, 8 * nw, hipMemcpyDeviceToHost);
      double mc = 0;
      for (auto v : h) mc += (double)v;
      mc /= nw;
      const double insts = 32.0 * ITER;  // per wave
      // per SIMD: wps waves, each `insts` instructions, over the wave's cycles
      printf("%-9s waves/SIMD %d: %.0f cycles per wave, %.3f instr/cycle/SIMD (%.3f per wave), "
             "kernel %.3f ms -> clock-free %.3f instr/ns/SIMD\n",
             names[mode], wps, mc, insts * wps / mc, insts / mc, ms,
             insts * nw / (ncu * 4.0) / (ms * 1e6));
    }
  }
  return 0;
}
