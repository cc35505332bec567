// Library identity, thread-local error reporting and the dropout step counter of the C ABI.
#include <cstdarg>
#include <cstdio>

#include "srf_common.h"
#include "../../include/srf.h"

namespace {
thread_local char g_err[512] = "";
thread_local const unsigned long long* t_seed_src = nullptr;
}

namespace srf {
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
const unsigned long long* seed_source() { return t_seed_src; }
}  // namespace srf

extern "C" {
int srf_version(void) { return 1; }

int srf_set_seed_source(const void* step_counter) {
  t_seed_src = static_cast<const unsigned long long*>(step_counter);
  return 0;
}
const char* srf_last_error(void) { return g_err; }
}
