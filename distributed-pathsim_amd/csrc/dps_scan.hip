// Device-wide exclusive prefix sum (reduce-then-scan), int64 output.
// Used for every CSR row pointer in the typed CSR build / SpGEMM / tile build.
#include "dps_common.hpp"

namespace dps {
namespace {

constexpr int kBlock = 256;
constexpr int kItems = 8;
constexpr int64_t kTile = kBlock * kItems;  // 2048 elements per block

template <class T>
__device__ __forceinline__ int64_t load_or0(const T* in, int64_t i, int64_t n) {
  return i < n ? static_cast<int64_t>(in[i]) : 0;
}

// Block-wide exclusive scan of one int64 per thread; returns exclusive prefix,
// *total = block sum.
__device__ int64_t block_exclusive(int64_t v, int64_t* lds_waves, int64_t* total) {
  const int lane = lane_id();
  const int wave = threadIdx.x / kWave;
  int64_t inc = wave_inclusive_sum(v);
  if (lane == kWave - 1) lds_waves[wave] = inc;
  __syncthreads();
  int64_t wave_off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kBlock / kWave; ++w) {
    int64_t s = lds_waves[w];
    if (w < wave) wave_off += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return wave_off + inc - v;
}

template <class T>
__global__ __launch_bounds__(kBlock) void k_block_reduce(const T* __restrict__ in, int64_t n,
                                                         int64_t* __restrict__ partial) {
  __shared__ int64_t lds[kBlock / kWave];
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kTile;
  int64_t s = 0;
#pragma unroll
  for (int i = 0; i < kItems; ++i) s += load_or0(in, base + i * kBlock + threadIdx.x, n);
  s = wave_sum(s);
  if (lane_id() == 0) lds[threadIdx.x / kWave] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t t = 0;
    for (int w = 0; w < kBlock / kWave; ++w) t += lds[w];
    partial[blockIdx.x] = t;
  }
}

// Scan of one tile with a per-block offset (offsets == nullptr -> 0).
template <class T>
__global__ __launch_bounds__(kBlock) void k_block_scan(const T* __restrict__ in, int64_t n,
                                                       const int64_t* __restrict__ offsets,
                                                       int64_t* __restrict__ out) {
  __shared__ int64_t lds[kBlock / kWave];
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kTile + threadIdx.x * kItems;
  int64_t v[kItems];
  int64_t s = 0;
#pragma unroll
  for (int i = 0; i < kItems; ++i) {
    v[i] = load_or0(in, base + i, n);
    s += v[i];
  }
  int64_t total;
  int64_t run = block_exclusive(s, lds, &total);
  if (offsets) run += offsets[blockIdx.x];
#pragma unroll
  for (int i = 0; i < kItems; ++i) {
    if (base + i < n) out[base + i] = run;
    run += v[i];
  }
  // out[n] = grand total: written by the thread that owns element n-1 (or n==0 case)
  if (n > 0 && base <= n - 1 && n - 1 < base + kItems) out[n] = run;
}

// The same scan whose block offset is the sum of the block reductions before
// it, read here (round 6: for up to kDirectBlocks blocks this replaces the
// separate single-block scan of the partial sums -- one launch fewer per scan,
// ~4.5 us each, nine scans per config3 build).
constexpr int64_t kDirectBlocks = 1024;
template <class T>
__global__ __launch_bounds__(kBlock) void k_block_scan_direct(const T* __restrict__ in, int64_t n,
                                                              const int64_t* __restrict__ partial,
                                                              int64_t* __restrict__ out) {
  __shared__ int64_t lds[kBlock / kWave];
  __shared__ int64_t off_s;
  int64_t o = 0;
  for (int64_t i = threadIdx.x; i < blockIdx.x; i += kBlock) o += partial[i];
  o = wave_sum(o);
  if (lane_id() == 0) lds[threadIdx.x / kWave] = o;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t t = 0;
    for (int w = 0; w < kBlock / kWave; ++w) t += lds[w];
    off_s = t;
  }
  __syncthreads();             // (lds is reused by block_exclusive)
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kTile + threadIdx.x * kItems;
  int64_t v[kItems];
  int64_t s = 0;
#pragma unroll
  for (int i = 0; i < kItems; ++i) {
    v[i] = load_or0(in, base + i, n);
    s += v[i];
  }
  int64_t total;
  int64_t run = block_exclusive(s, lds, &total) + off_s;
#pragma unroll
  for (int i = 0; i < kItems; ++i) {
    if (base + i < n) out[base + i] = run;
    run += v[i];
  }
  if (n > 0 && base <= n - 1 && n - 1 < base + kItems) out[n] = run;
}

__global__ void k_zero_total(int64_t* out) { out[0] = 0; }

}  // namespace

size_t scan_workspace_size(int64_t n) {
  size_t total = 0;
  int64_t m = n;
  while (m > kTile) {
    int64_t nb = (m + kTile - 1) / kTile;
    total += align_up(static_cast<size_t>(nb) * sizeof(int64_t));       // partial sums
    total += align_up(static_cast<size_t>(nb + 1) * sizeof(int64_t));   // their scan
    m = nb;
  }
  return total + 256;
}

template <class T>
hipError_t scan_exclusive(const T* in, int64_t* out, int64_t n, void* ws, size_t ws_bytes,
                          hipStream_t stream) {
  if (n <= 0) {
    k_zero_total<<<1, 1, 0, stream>>>(out);
    return hipGetLastError();
  }
  const int64_t nb = (n + kTile - 1) / kTile;
  if (nb == 1) {
    k_block_scan<T><<<1, kBlock, 0, stream>>>(in, n, nullptr, out);
    return hipGetLastError();
  }
  Carve c(ws, ws_bytes);
  int64_t* partial = c.take<int64_t>(nb);
  int64_t* pscan = c.take<int64_t>(nb + 1);
  if (!c.ok) return hipErrorInvalidValue;
  k_block_reduce<T><<<static_cast<unsigned>(nb), kBlock, 0, stream>>>(in, n, partial);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (nb <= kDirectBlocks) {
    k_block_scan_direct<T><<<static_cast<unsigned>(nb), kBlock, 0, stream>>>(in, n, partial, out);
    return hipGetLastError();
  }
  e = scan_exclusive<int64_t>(partial, pscan, nb, c.base + c.off, c.cap - c.off, stream);
  if (e != hipSuccess) return e;
  k_block_scan<T><<<static_cast<unsigned>(nb), kBlock, 0, stream>>>(in, n, pscan, out);
  return hipGetLastError();
}

template hipError_t scan_exclusive<int32_t>(const int32_t*, int64_t*, int64_t, void*, size_t,
                                            hipStream_t);
template hipError_t scan_exclusive<uint32_t>(const uint32_t*, int64_t*, int64_t, void*, size_t,
                                             hipStream_t);
template hipError_t scan_exclusive<int64_t>(const int64_t*, int64_t*, int64_t, void*, size_t,
                                            hipStream_t);

namespace {
__global__ __launch_bounds__(256) void k_fill_set(FillSet s) {
  for (int r = 0; r < s.k; ++r) {
    uint32_t* __restrict__ p = s.p[r];
    const uint32_t v = s.v[r];
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < s.n[r];
         i += static_cast<int64_t>(gridDim.x) * 256)
      p[i] = v;
  }
}
}  // namespace

hipError_t fill_set(const FillSet& s, hipStream_t stream) {
  if (s.overflow) return hipErrorInvalidValue;   // more ranges than FillSet::kMax
  if (s.k == 0) return hipSuccess;
  int64_t longest = 1;
  for (int r = 0; r < s.k; ++r) longest = s.n[r] > longest ? s.n[r] : longest;
  const int64_t blocks = (longest + 255) / 256;
  k_fill_set<<<static_cast<unsigned>(blocks < 4096 ? blocks : 4096), 256, 0, stream>>>(s);
  return hipGetLastError();
}

}  // namespace dps
