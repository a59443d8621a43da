// UTF-8 validation of a device text buffer: the strict decode that dask.bag.read_text applies
// to every input block (the reference raises UnicodeDecodeError on malformed input), done on the
// bytes the GPU is about to process instead of decoding the whole corpus into Python strings.
//
// Python's UTF-8 decoder (Objects/stringlib/codecs.h) accepts exactly the well-formed sequences
// of Unicode 3.2+ table 3-7: 00-7F | C2-DF 80-BF | E0 A0-BF 80-BF | E1-EC 80-BF 80-BF |
// ED 80-9F 80-BF | EE-EF 80-BF 80-BF | F0 90-BF 80-BF 80-BF | F1-F3 80-BF 80-BF 80-BF |
// F4 80-8F 80-BF 80-BF. Each thread checks the sequences that START in its 16-byte slice (a
// continuation byte is never a start, so every byte is covered by exactly one start; a
// continuation with no covering lead is caught as a stray) and reports the first bad offset.
#include "common.h"
#include "device.h"
#include "lddl_amd.h"

namespace lddl {
namespace {

// length of the well-formed sequence starting at p[0] (<= 4 bytes available: n), 0 if malformed
__device__ inline int seq_len(const uint8_t* p, int64_t n) {
  const uint32_t c = p[0];
  if (c < 0x80) return 1;
  int len;
  uint32_t lo = 0x80, hi = 0xBF;
  if (c >= 0xC2 && c <= 0xDF) len = 2;
  else if (c >= 0xE0 && c <= 0xEF) {
    len = 3;
    if (c == 0xE0) lo = 0xA0;
    if (c == 0xED) hi = 0x9F;
  } else if (c >= 0xF0 && c <= 0xF4) {
    len = 4;
    if (c == 0xF0) lo = 0x90;
    if (c == 0xF4) hi = 0x8F;
  } else {
    return 0;  // continuation byte, C0/C1 or F5-FF as a lead
  }
  if (n < len) return 0;
  if (p[1] < lo || p[1] > hi) return 0;
  for (int k = 2; k < len; ++k)
    if ((p[k] & 0xC0) != 0x80) return 0;
  return len;
}

constexpr int kSlice = 16;

__global__ void __launch_bounds__(256) utf8_check_kernel(const uint8_t* __restrict__ text, int64_t n,
                                                         unsigned long long* __restrict__ first_bad) {
  const int64_t s0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * kSlice;
  if (s0 >= n) return;
  const int64_t s1 = s0 + kSlice < n ? s0 + kSlice : n;
  // the sequence covering s0 may have started up to 3 bytes earlier: find this slice's first start
  int64_t i = s0;
  if (i > 0 && (text[i] & 0xC0) == 0x80) {
    int64_t j = i - 1;
    while (j > 0 && j > i - 3 && (text[j] & 0xC0) == 0x80) --j;
    const int l = seq_len(text + j, n - j);
    if (l > 0 && j + l > i) i = j + l;  // continuation of a well-formed sequence: skip it
    // otherwise text[i] is a stray continuation byte: reported below as a bad start
  }
  for (; i < s1;) {
    const int l = seq_len(text + i, n - i);
    if (l == 0) {
      atomicMin(first_bad, (unsigned long long)i);
      return;
    }
    i += l;
  }
}

}  // namespace
}  // namespace lddl

using namespace lddl;

extern "C" int lddl_utf8_check(void* stream, const uint8_t* d_text, int64_t n_bytes,
                               int64_t* d_first_bad) {
  if (!d_first_bad || n_bytes < 0) LDDL_FAIL(-1, "bad arguments");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  LDDL_HIP(hipMemsetAsync(d_first_bad, 0x7F, sizeof(int64_t), st));  // > any offset
  if (n_bytes == 0) return 0;
  const int64_t threads = (n_bytes + kSlice - 1) / kSlice;
  hipLaunchKernelGGL(utf8_check_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st,
                     d_text, n_bytes, reinterpret_cast<unsigned long long*>(d_first_bad));
  LDDL_HIP(hipGetLastError());
  return 0;
}
