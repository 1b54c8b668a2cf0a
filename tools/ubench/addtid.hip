// Probe: does ds_write_addtid_b32 (M0 + offset + 4*lane) address the issuing
// workgroup's own LDS allocation when many one-wave workgroups share a CU?
// And its zeroing rate against ds_write_b128 (cycles per 8 KiB).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ void addtid_1k(uint32_t base_bytes, uint32_t v) {
  uint32_t save;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"   // SALU write of M0 -> LDS add-TID: one wait state
      "ds_write_addtid_b32 %2 offset:0\n\t"
      "ds_write_addtid_b32 %2 offset:256\n\t"
      "ds_write_addtid_b32 %2 offset:512\n\t"
      "ds_write_addtid_b32 %2 offset:768\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(save) : "s"(base_bytes), "v"(v) : "memory");
}

__global__ __launch_bounds__(64) void k_check(uint32_t* bad, uint32_t* first) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[2048];
  const int lane = threadIdx.x;
  for (int i = lane; i < 2048; i += 64) lds[i] = 0xAAAA0000u | blockIdx.x;
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  const uint32_t base = __builtin_amdgcn_readfirstlane(1024u * (blockIdx.x & 3));   // bytes
  addtid_1k(base, blockIdx.x + 1);
  __builtin_amdgcn_wave_barrier();
  uint32_t nb = 0;
  for (int i = lane; i < 2048; i += 64) {
    const bool in = i * 4 >= (int)base && i * 4 < (int)base + 1024;
    const uint32_t want = in ? blockIdx.x + 1 : (0xAAAA0000u | blockIdx.x);
    if (lds[i] != want) { ++nb; if (first[blockIdx.x] == 0) first[blockIdx.x] = lds[i] | 1u; }
  }
  atomicAdd(&bad[blockIdx.x], nb);
}

__global__ __launch_bounds__(64) void k_rate(int iters, int mode, uint64_t* cyc, uint32_t* sink) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[2048];
  const int lane = threadIdx.x;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (mode == 0) {
#pragma unroll
      for (int b = 0; b < 2048; b += 256)
        *reinterpret_cast<uint4*>(lds + b + lane * 4) = make_uint4(it, 0, 0, 0);
    } else {
#pragma unroll
      for (int b = 0; b < 8; ++b) addtid_1k(b * 1024u, it);
    }
    __builtin_amdgcn_s_waitcnt(0);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
  sink[blockIdx.x * 64 + lane] = lds[lane * 31];
}

int main() {
  int dev = 0, ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int nb = ncu * 20;
  uint32_t *bad, *first, *sink;
  uint64_t* cyc;
  CK(hipMalloc(&bad, nb * 4)); CK(hipMalloc(&first, nb * 4)); CK(hipMalloc(&sink, nb * 256)); CK(hipMalloc(&cyc, nb * 8));
  CK(hipMemset(bad, 0, nb * 4)); CK(hipMemset(first, 0, nb * 4));
  k_check<<<nb, 64>>>(bad, first);
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> hb(nb), hf(nb);
  CK(hipMemcpy(hb.data(), bad, nb * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hf.data(), first, nb * 4, hipMemcpyDeviceToHost));
  long tot = 0; int nbad = 0;
  for (int i = 0; i < nb; ++i) { tot += hb[i]; if (hb[i]) { if (nbad < 4) printf("block %d: %u bad dwords, first value 0x%08x\n", i, hb[i], hf[i]); ++nbad; } }
  printf("addtid check: %d of %d blocks wrong, %ld bad dwords\n", nbad, nb, tot);
  for (int mode = 0; mode < 2; ++mode) {
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const int iters = 20000;
    k_rate<<<nb, 64>>>(100, mode, cyc, sink);
    hipEventRecord(e0);
    k_rate<<<nb, 64>>>(iters, mode, cyc, sink);
    hipEventRecord(e1);
    CK(hipDeviceSynchronize());
    float ms = 0; hipEventElapsedTime(&ms, e0, e1);
    const double bytes = double(nb) * iters * 8192.0;
    printf("%s: %.3f ms, %.1f TB/s zeroed, %.1f B/clk/CU at 2.4 GHz\n", mode ? "ds_write_addtid_b32" : "ds_write_b128",
           ms, bytes / ms / 1e9, bytes / (ms * 1e-3) / (ncu * 2.4e9));
  }
  return 0;
}
