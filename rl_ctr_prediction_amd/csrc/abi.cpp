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

extern "C" int ctr_abi_version(void) { return 13; }

extern "C" const char* ctr_last_error(void) { return ctr::g_last_error; }

extern "C" int ctr_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

extern "C" int ctr_stream_create_cu_masked(const uint32_t* mask, int n_words, ctr_stream_t* out) {
  if (!mask || n_words <= 0 || !out) {
    ctr::set_error("ctr_stream_create_cu_masked: null mask / output or n_words <= 0");
    return CTR_ERR_INVALID;
  }
  hipStream_t s = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)n_words, mask);
  if (e != hipSuccess) {
    ctr::set_error("hipExtStreamCreateWithCUMask: %s", hipGetErrorString(e));
    return CTR_ERR_HIP;
  }
  *out = s;
  return CTR_OK;
}

extern "C" int ctr_stream_destroy(ctr_stream_t stream) {
  const hipError_t e = hipStreamDestroy(static_cast<hipStream_t>(stream));
  if (e != hipSuccess) {
    ctr::set_error("hipStreamDestroy: %s", hipGetErrorString(e));
    return CTR_ERR_HIP;
  }
  return CTR_OK;
}
