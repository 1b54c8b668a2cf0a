// Microbenchmarks for the hot kernel's primitives on gfx950:
//  1. no-return ds_add_u32 at random dwords of a W/4-dword LDS buffer
//  2. 16-byte global loads of random chunks of a 32 MB buffer (MALL resident)
//  3. both combined (load chunk -> 4 adds)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint32_t xs(uint32_t& s) { s ^= s << 13; s ^= s >> 17; s ^= s << 5; return s; }

__global__ __launch_bounds__(256) void k_lds_add(int iters, int ndw, uint32_t* out) {
  extern __shared__ uint32_t acc[];
  for (int i = threadIdx.x; i < ndw; i += 256) acc[i] = 0;
  __syncthreads();
  uint32_t s = 0x9E3779B9u * (blockIdx.x * 256 + threadIdx.x + 1);
  const uint32_t mask = ndw - 1;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const uint32_t r = xs(s);
      __hip_atomic_fetch_add(&acc[r & mask], 1u << ((r >> 27) & 24), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = acc[blockIdx.x & mask];
}

__global__ __launch_bounds__(256) void k_gload(int iters, const uint4* __restrict__ buf, uint32_t nchunk, uint32_t* out) {
  uint32_t s = 0x9E3779B9u * (blockIdx.x * 256 + threadIdx.x + 1);
  uint32_t x = 0;
  for (int it = 0; it < iters; ++it) {
    uint4 v[4];
    // consecutive lanes read consecutive chunks (coalesced 1 KB per wave instr)
    const uint32_t base = (xs(s) & (nchunk - 1)) & ~255u;
    const uint32_t b0 = __builtin_amdgcn_readfirstlane(base);
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = buf[(b0 + u * 256 + threadIdx.x) & (nchunk - 1)];
#pragma unroll
    for (int u = 0; u < 4; ++u) x += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (x == 0x12345678u) out[0] = x;
}

__global__ __launch_bounds__(256) void k_both(int iters, const uint4* __restrict__ buf, uint32_t nchunk, int ndw, uint32_t* out) {
  extern __shared__ uint32_t acc[];
  for (int i = threadIdx.x; i < ndw; i += 256) acc[i] = 0;
  __syncthreads();
  uint32_t s = 0x9E3779B9u * (blockIdx.x * 256 + threadIdx.x + 1);
  const uint32_t mask = (ndw - 1) << 2;
  for (int it = 0; it < iters; ++it) {
    uint4 v[4];
    const uint32_t base = __builtin_amdgcn_readfirstlane((xs(s) & (nchunk - 1)) & ~255u);
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = buf[(base + u * 256 + threadIdx.x) & (nchunk - 1)];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      uint32_t e[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        __hip_atomic_fetch_add(&acc[(e[j] & mask) >> 2], (e[j] >> 16) << ((e[j] << 3) & 24), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = acc[blockIdx.x & (ndw - 1)];
}

int main() {
  int dev; CK(hipGetDevice(&dev));
  int ncu; CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  int clk; CK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev));
  printf("CUs %d clock %d kHz\n", ncu, clk);
  uint32_t* out; CK(hipMalloc(&out, 1 << 20));
  const uint32_t nchunk = 2u << 20;   // 32 MB of 16-B chunks
  uint4* buf; CK(hipMalloc(&buf, (size_t)nchunk * 16));
  std::vector<uint32_t> h((size_t)nchunk * 4);
  uint32_t s = 1;
  for (auto& x : h) { s ^= s << 13; s ^= s >> 17; s ^= s << 5; x = s & 0x00FFFFFFu; }
  CK(hipMemcpy(buf, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  float ms;
  for (int wpc : {2, 4, 8}) {
    for (int ndw : {1024, 4096, 8192}) {
      const int lds = ndw * 4;
      CK(hipFuncSetAttribute((const void*)k_lds_add, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
      const int grid = ncu * wpc, iters = 2000;
      k_lds_add<<<grid, 256, lds>>>(10, ndw, out);
      CK(hipEventRecord(a)); k_lds_add<<<grid, 256, lds>>>(iters, ndw, out); CK(hipEventRecord(b));
      CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
      double adds = (double)grid * 256 * iters * 16;
      printf("lds_add  wg/cu %d dwords %5d: %.2f ms  %.3e adds/s  %.2f adds/clk/CU\n", wpc, ndw, ms, adds / ms * 1e3,
             adds / (ms * 1e-3) / ncu / (clk * 1e3));
    }
  }
  for (int wpc : {2, 4, 8}) {
    const int grid = ncu * wpc, iters = 2000;
    k_gload<<<grid, 256>>>(10, buf, nchunk, out);
    CK(hipEventRecord(a)); k_gload<<<grid, 256>>>(iters, buf, nchunk, out); CK(hipEventRecord(b));
    CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
    double bytes = (double)grid * 256 * iters * 64;
    printf("gload    wg/cu %d: %.2f ms  %.1f GB/s  %.1f B/clk/CU\n", wpc, ms, bytes / ms * 1e-6,
           bytes / (ms * 1e-3) / ncu / (clk * 1e3));
  }
  for (int wpc : {2, 4, 8}) {
    const int ndw = 4096, lds = ndw * 4;
    CK(hipFuncSetAttribute((const void*)k_both, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    const int grid = ncu * wpc, iters = 2000;
    k_both<<<grid, 256, lds>>>(10, buf, nchunk, ndw, out);
    CK(hipEventRecord(a)); k_both<<<grid, 256, lds>>>(iters, buf, nchunk, ndw, out); CK(hipEventRecord(b));
    CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
    double terms = (double)grid * 256 * iters * 16;
    printf("both     wg/cu %d: %.2f ms  %.3e terms/s  %.2f terms/clk/CU\n", wpc, ms, terms / ms * 1e3,
           terms / (ms * 1e-3) / ncu / (clk * 1e3));
  }
  return 0;
}
