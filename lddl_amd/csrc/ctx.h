// Host-side context: device copies of the normaliser table and the vocab hash.
#pragma once
#include <hip/hip_runtime.h>
#include <string>
#include <vector>

#include "device.h"

struct lddl_ctx {
  int device = 0;
  lddl::Tables tab{};
  // owned device allocations
  uint16_t* d_l1 = nullptr;
  uint32_t* d_pages = nullptr;
  uint8_t* d_pool = nullptr;
  lddl::VEnt* d_vhash = nullptr;
  uint8_t* d_vbytes = nullptr;
  int64_t* d_voff = nullptr;
  uint8_t* d_render = nullptr;      // full token strings (as in vocab.txt, "##" kept)
  int64_t* d_render_off = nullptr;  // token i = d_render[off[i] .. off[i+1])
  uint32_t* d_bloom = nullptr;
  int32_t vocab_size = 0;
  std::vector<std::string> tokens;  // host copy of the vocab lines
};

namespace lddl {
inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
}  // namespace lddl
