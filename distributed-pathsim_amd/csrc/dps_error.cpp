// C-ABI plumbing without HIP: thread-local error text and the ABI version.
#include <cstdarg>
#include <cstdio>

#include "dps_host.hpp"

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
}
