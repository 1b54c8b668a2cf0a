// Host-only error plumbing shared by every translation unit of libdpathsim
// (no HIP headers: dps_log.cpp and the sanitizer builds use it alone).
#pragma once

#include "dpathsim.h"

namespace dps {
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
// current dps_set_tuning value of `key` (0 = automatic)
int tuning(int key);
}  // namespace dps

#define DPS_REQUIRE(cond, code, ...)                                                   \
  do {                                                                                 \
    if (!(cond)) {                                                                     \
      dps::set_error(__VA_ARGS__);                                                     \
      return (code);                                                                   \
    }                                                                                  \
  } while (0)
