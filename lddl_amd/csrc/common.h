// Shared host-side helpers: thread-local error reporting and HIP call checking.
#pragma once
#include <cstdarg>
#include <cstdio>
#include <string>

namespace lddl {
void set_error(const char* fmt, ...);
}  // namespace lddl

#define LDDL_FAIL(code, ...)              \
  do {                                    \
    ::lddl::set_error(__VA_ARGS__);       \
    return (code);                        \
  } while (0)

#define LDDL_HIP(expr)                                                                    \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      LDDL_FAIL(-100, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
  } while (0)
