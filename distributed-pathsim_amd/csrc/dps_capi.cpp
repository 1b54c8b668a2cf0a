// C-ABI plumbing that needs the HIP runtime: the device count.
#include <hip/hip_runtime.h>

#include "dps_host.hpp"

extern "C" {
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
