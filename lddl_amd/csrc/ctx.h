// Host-side context: device copies of the normaliser table and the vocab hash.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include <algorithm>
#include <mutex>

#include "device.h"

namespace lddl {
// Device memory cache for the library's per-call temporaries (pair plans). Blocks are plain
// hipMalloc allocations that are never returned while the context lives: a released block goes
// to the free list with an event recorded on the releasing stream, and a later request takes the
// smallest free block that fits (up to 1.5x the request; a stream other than the releasing one
// waits on the event first). A batch-per-step workload therefore allocates only in its first
// step. (The stream-ordered HIP pool that this replaces showed 0.4-2 s hipMallocAsync calls
// once torch's caching allocator held a large share of HBM.)
//
// With an external allocator set (lddl_ctx_set_allocator: the host hands in its own device
// allocator, e.g. PyTorch's caching allocator), blocks come from and go straight back to it and
// nothing is cached here, so one pool owns HBM.
class DevArena {
 public:
  typedef void* (*AllocFn)(size_t bytes, void* stream, void* user);
  typedef void (*FreeFn)(void* p, void* stream, void* user);
  struct Block {
    void* p = nullptr;
    size_t size = 0;
    hipEvent_t ev = nullptr;
    hipStream_t st = nullptr;
    bool ext = false;  // from the external allocator
  };
  void set_external(AllocFn a, FreeFn f, void* user) {
    trim();
    std::lock_guard<std::mutex> g(mu_);
    alloc_ = a;
    free_fn_ = f;
    user_ = user;
  }
  hipError_t take(size_t bytes, hipStream_t st, Block& out) {
    if (alloc_) {
      out = Block{};
      out.size = bytes ? bytes : 16;
      out.p = alloc_(out.size, (void*)st, user_);
      out.ext = true;
      out.st = st;
      return out.p ? hipSuccess : hipErrorOutOfMemory;
    }
    const size_t want = round_up(bytes);
    {
      std::lock_guard<std::mutex> g(mu_);
      size_t best = free_.size();
      for (size_t i = 0; i < free_.size(); ++i)
        if (free_[i].size >= want && free_[i].size <= want + want / 2 &&
            (best == free_.size() || free_[i].size < free_[best].size))
          best = i;
      if (best < free_.size()) {
        out = free_[best];
        free_.erase(free_.begin() + (ptrdiff_t)best);
        if (out.st != st && out.ev) (void)hipStreamWaitEvent(st, out.ev, 0);
        return hipSuccess;
      }
    }
    out = Block{};
    out.size = want;
    hipError_t e = hipMalloc(&out.p, want);
    if (e != hipSuccess) {  // release the cached blocks and retry once
      (void)hipGetLastError();
      trim();
      e = hipMalloc(&out.p, want);
    }
    return e;
  }
  void give(Block b, hipStream_t st) {
    if (!b.p) return;
    if (b.ext) {
      // a stream-ordered external pool (torch's caching allocator) reuses the block on the stream
      // it was allocated on: when the last use was on another stream, that stream is ordered
      // after it first, so no later allocation there can overwrite the block while it is in use
      if (st != b.st) {
        hipEvent_t ev;
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess) {
          (void)hipEventRecord(ev, st);
          (void)hipStreamWaitEvent(b.st, ev, 0);
          (void)hipEventDestroy(ev);
        }
      }
      if (free_fn_) free_fn_(b.p, (void*)b.st, user_);
      return;
    }
    if (!b.ev) (void)hipEventCreateWithFlags(&b.ev, hipEventDisableTiming);
    if (b.ev) (void)hipEventRecord(b.ev, st);
    b.st = st;
    std::lock_guard<std::mutex> g(mu_);
    free_.push_back(b);
  }
  void trim() {  // free every cached block (after the work that used them)
    std::lock_guard<std::mutex> g(mu_);
    for (Block& b : free_) {
      if (b.ev) {
        (void)hipEventSynchronize(b.ev);
        (void)hipEventDestroy(b.ev);
      }
      (void)hipFree(b.p);
    }
    free_.clear();
  }
  ~DevArena() { trim(); }

 private:
  static size_t round_up(size_t b) {  // 2 MiB granules, 1/16 of the size above 32 MiB
    size_t g = (size_t)2 << 20;
    if (b > ((size_t)32 << 20)) g = std::max(g, b / 16);
    return (b + g - 1) / g * g;
  }
  std::mutex mu_;
  std::vector<Block> free_;
  AllocFn alloc_ = nullptr;
  FreeFn free_fn_ = nullptr;
  void* user_ = nullptr;
};

// A temporary from the arena for the duration of one C-ABI call (returned on `st`).
struct ArenaTmp {
  DevArena* a;
  hipStream_t st;
  DevArena::Block b{};
  ArenaTmp(DevArena* arena, hipStream_t stream) : a(arena), st(stream) {}
  hipError_t take(size_t bytes) { return a->take(bytes, st, b); }
  template <typename T>
  T* as() const { return static_cast<T*>(b.p); }
  ~ArenaTmp() { a->give(b, st); }
};
}  // namespace lddl

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
  uint64_t* d_vlong = nullptr;
  int32_t vocab_size = 0;
  // bytes per token id in the pair tables (dense kept tokens, sample tokens, labels): 2 when every
  // id fits uint16 with two values to spare for the gather's decision table (vocab_size <=
  // 65,534: BERT's uncased 30,522 and cased 28,996), else 4
  int32_t id_bytes() const { return vocab_size <= 65534 ? 2 : 4; }
  size_t lds_per_block = 0;         // hipDeviceAttributeMaxSharedMemoryPerBlock of `device`
  std::vector<std::string> tokens;  // host copy of the vocab lines
  lddl::DevArena arena;             // per-call temporaries (pair plans)
  void* punkt = nullptr;            // lddl_punkt_state (segment.hip), created by lddl_punkt_set_params
};
extern "C" void lddl_punkt_release(lddl_ctx* c);

namespace lddl {
inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
}  // namespace lddl
