// Library-level C ABI entry points: version, thread-local error text, device probe.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "../../include/ctr_hip.h"

namespace ctr {

static thread_local char g_last_error[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}

}  // namespace ctr

extern "C" int ctr_abi_version(void) { return 12; }

extern "C" const char* ctr_last_error(void) { return ctr::g_last_error; }

extern "C" int ctr_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
