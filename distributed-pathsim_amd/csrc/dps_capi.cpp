// C-ABI plumbing that needs the HIP runtime: the device count; the explicit
// tuning overrides (dps_set_tuning) the kernels consult.
#include <hip/hip_runtime.h>

#include <atomic>

#include "dps_host.hpp"

namespace dps {
namespace {
std::atomic<int> g_tune[DPS_TUNE_KEYS];
}
int tuning(int key) { return key > 0 && key < DPS_TUNE_KEYS ? g_tune[key].load() : 0; }
}  // namespace dps

extern "C" {
int dps_set_tuning(int32_t key, int32_t value) {
  DPS_REQUIRE(key > 0 && key < DPS_TUNE_KEYS, DPS_ERR_INVALID, "unknown tuning key %d", key);
  if (key == DPS_TUNE_WAVES_PER_ROW)
    DPS_REQUIRE(value == 0 || value == 1 || value == 4 || value == 8, DPS_ERR_INVALID,
                "waves per row must be 0 (automatic), 1, 4 or 8, got %d", value);
  if (key == DPS_TUNE_TILE_BUILD)
    DPS_REQUIRE(value >= 0 && value <= 2, DPS_ERR_INVALID,
                "tile build must be 0 (automatic), 1 (block-local) or 2 (global atomics), got %d",
                value);
  if (key == DPS_TUNE_BANK_ORDER)
    DPS_REQUIRE(value >= 0 && value <= 2, DPS_ERR_INVALID,
                "bank order must be 0 (automatic), 1 (on) or 2 (off), got %d", value);
  if (key == DPS_TUNE_LEAN_WPC)
    DPS_REQUIRE(value >= 0 && value <= 32, DPS_ERR_INVALID,
                "workgroups per CU must be 0 (automatic) or 1..32, got %d", value);
  dps::g_tune[key].store(value);
  return DPS_OK;
}
int dps_get_tuning(int32_t key) { return dps::tuning(key); }

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
