#include "common.h"
#include "lddl_amd.h"

namespace lddl {
static thread_local std::string g_err;
void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
}
}  // namespace lddl

extern "C" const char* lddl_last_error(void) { return lddl::g_err.c_str(); }
extern "C" int lddl_version(void) { return 1; }
