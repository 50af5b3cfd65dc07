// Library-level C ABI: version and the thread-local error string.
#include <cstdarg>
#include <cstdio>

#include "common.hpp"

namespace tt {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace tt

extern "C" int tt_version(void) { return 1; }
extern "C" const char* tt_last_error(void) { return tt::g_err; }
