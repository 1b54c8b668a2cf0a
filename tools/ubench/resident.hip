// Probe (round 6): how many one-wave workgroups are resident on a CU at once
// for the hot kernel's resource shape (8 KiB of LDS, 96 VGPRs, ~106 SGPRs)?
// The profiling build's wave stamps showed 512 of k_cct1's 5120 workgroups
// (two per CU) starting only at the end of the launch.  Each variant launches
// 20 workgroups per CU that record their realtime start, touch their LDS and
// spin for SPIN_US; the count that started within the first 10 % of the spin
// is the resident capacity.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      printf("%s: %s\n", #x, hipGetErrorString(e));                              \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

constexpr int kSpinTicks = 100 * 2000;   // 2 ms at the 100 MHz realtime clock

// VG: force the VGPR allocation with a clobber of v(VG-1); SG: of s(SG-1).
template <int VG, int SG>
__global__ __launch_bounds__(64) void k_resident(unsigned long long* t) {
  extern __shared__ uint32_t lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) t[blockIdx.x] = t0;
  lds[threadIdx.x] = threadIdx.x;
  if constexpr (VG == 96) asm volatile("v_mov_b32 v95, 0" ::: "v95");
  if constexpr (VG == 80) asm volatile("v_mov_b32 v79, 0" ::: "v79");
  if constexpr (VG == 104) asm volatile("v_mov_b32 v103, 0" ::: "v103");
  if constexpr (SG == 102) asm volatile("s_mov_b32 s101, 0" ::: "s101");
  if constexpr (SG == 90) asm volatile("s_mov_b32 s89, 0" ::: "s89");
  while (__builtin_amdgcn_s_memrealtime() - t0 < kSpinTicks) __builtin_amdgcn_s_sleep(10);
  if (lds[(threadIdx.x + 1) & 63] == 12345u) t[blockIdx.x] = 0;   // keep the LDS live
}

template <int VG, int SG>
int run(const char* name, size_t lds_bytes, int wpc, int n_cu, unsigned long long* d_t) {
  const int grid = wpc * n_cu;
  CK(hipMemset(d_t, 0, grid * sizeof(unsigned long long)));
  k_resident<VG, SG><<<grid, 64, lds_bytes>>>(d_t);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> t(grid);
  CK(hipMemcpy(t.data(), d_t, grid * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  const unsigned long long t0 = *std::min_element(t.begin(), t.end());
  int early = 0;
  for (unsigned long long v : t) early += (v - t0) < kSpinTicks / 10 ? 1 : 0;
  printf("%-34s lds %6zu B  %2d WG/CU launched: %5d of %5d started at once (%.2f per CU)\n", name,
         lds_bytes, wpc, early, grid, static_cast<double>(early) / n_cu);
  return 0;
}

int main() {
  int dev = 0, n_cu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
  unsigned long long* d_t = nullptr;
  CK(hipMalloc(&d_t, 64 * n_cu * sizeof(unsigned long long)));
  printf("%d CUs\n", n_cu);
  int rc = 0;
  rc |= run<8, 0>("few VGPRs, 8 KiB LDS", 8192, 20, n_cu, d_t);
  for (size_t b : {7712, 7744, 7808, 7936, 8064, 8128, 8160})
    rc |= run<8, 0>("few VGPRs", b, 20, n_cu, d_t);
  rc |= run<8, 0>("few VGPRs, 16 KiB LDS", 16384, 12, n_cu, d_t);
  rc |= run<8, 0>("few VGPRs, 15.5 KiB LDS", 15872, 12, n_cu, d_t);
  rc |= run<8, 0>("few VGPRs, 32 KiB LDS", 32768, 6, n_cu, d_t);
  rc |= run<8, 0>("few VGPRs, 7.5 KiB LDS", 7680, 20, n_cu, d_t);
  rc |= run<8, 0>("few VGPRs, 4 KiB LDS", 4096, 24, n_cu, d_t);
  rc |= run<8, 0>("few VGPRs, no LDS", 0, 32, n_cu, d_t);
  rc |= run<96, 0>("96 VGPRs, no LDS", 0, 24, n_cu, d_t);
  rc |= run<96, 0>("96 VGPRs, 8 KiB LDS", 8192, 20, n_cu, d_t);
  rc |= run<96, 102>("96 VGPRs, 102 SGPRs, 8 KiB LDS", 8192, 20, n_cu, d_t);
  rc |= run<96, 102>("96 VGPRs, 102 SGPRs, no LDS", 0, 24, n_cu, d_t);
  rc |= run<8, 102>("few VGPRs, 102 SGPRs, no LDS", 0, 32, n_cu, d_t);
  rc |= run<8, 90>("few VGPRs, 90 SGPRs, no LDS", 0, 32, n_cu, d_t);
  rc |= run<80, 0>("80 VGPRs, 8 KiB LDS", 8192, 20, n_cu, d_t);
  rc |= run<96, 90>("96 VGPRs, 90 SGPRs, 8 KiB LDS", 8192, 20, n_cu, d_t);
  CK(hipFree(d_t));
  return rc;
}
