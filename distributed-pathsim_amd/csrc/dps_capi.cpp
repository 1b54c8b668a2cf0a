// C-ABI plumbing: thread-local error text, version, device count.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>

#include "dpathsim.h"

namespace dps {
namespace {
thread_local char g_err[1024] = "";
}
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace dps

extern "C" {
int dps_abi_version(void) { return DPS_ABI_VERSION; }
const char* dps_last_error(void) { return dps::g_err; }
int dps_device_count(void) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    dps::set_error("hipGetDeviceCount: %s", hipGetErrorString(e));
    return DPS_ERR_HIP;
  }
  return n;
}
}
