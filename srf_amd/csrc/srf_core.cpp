// Library identity and thread-local error reporting for the C ABI.
#include <cstdarg>
#include <cstdio>

#include "srf_common.h"
#include "../../include/srf.h"

namespace {
thread_local char g_err[512] = "";
}

namespace srf {
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace srf

extern "C" {
int srf_version(void) { return 1; }
const char* srf_last_error(void) { return g_err; }
}
