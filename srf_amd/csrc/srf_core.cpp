// Library identity, thread-local error reporting and the dropout step counter of the C ABI.
#include <atomic>
#include <cstdarg>
#include <cstdio>

#include "srf_common.h"
#include "../../include/srf.h"

namespace {
thread_local char g_err[512] = "";
// Process-global, not thread-local: torch runs the autograd backward of device
// tensors on its own per-device worker thread, and the backward kernels must
// rebuild the forward's dropout masks from the same counter.
std::atomic<const unsigned long long*> g_seed_src{nullptr};
std::atomic<unsigned*> g_fault{nullptr};
}

namespace srf {
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
const unsigned long long* seed_source() { return g_seed_src.load(std::memory_order_acquire); }
unsigned* fault_flag() { return g_fault.load(std::memory_order_acquire); }
}  // namespace srf

extern "C" {
int srf_version(void) { return 1; }

int srf_set_seed_source(const void* step_counter) {
  g_seed_src.store(static_cast<const unsigned long long*>(step_counter), std::memory_order_release);
  return 0;
}
int srf_set_fault_flag(void* flag) {
  g_fault.store(static_cast<unsigned*>(flag), std::memory_order_release);
  return 0;
}
const char* srf_last_error(void) { return g_err; }
}
