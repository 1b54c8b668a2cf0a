// Stable LSD radix sort of (uint64 key, uint32 value) pairs, 8-bit digits.
// Used to relabel PathSim targets in ascending global-walk order (see
// dps_target_order in dps_topk.hip): a pure layout step -- results never
// depend on the order, only the hot kernel's pruning efficiency does.
#include "dps_common.hpp"

namespace dps {
namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / kWave;
constexpr int kItems = 16;
constexpr int kTile = kBlock * kItems;  // 4096 keys per block
constexpr int kRadix = 256;

__global__ __launch_bounds__(kBlock) void k_radix_hist(const uint64_t* __restrict__ keys,
                                                       int64_t n, int shift,
                                                       uint32_t* __restrict__ hist,
                                                       int64_t nblocks) {
  __shared__ uint32_t h[kRadix];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kTile;
#pragma unroll 4
  for (int r = 0; r < kItems; ++r) {
    const int64_t i = base + r * kBlock + threadIdx.x;
    if (i < n) atomicAdd(&h[(keys[i] >> shift) & 0xFF], 1u);
  }
  __syncthreads();
  hist[static_cast<int64_t>(threadIdx.x) * nblocks + blockIdx.x] = h[threadIdx.x];
}

// Stable scatter, staged through LDS: the tile is consumed in kItems rounds
// of 256 keys in index order; inside a round keys are ranked by (wave, lane)
// with per-wave multi-split ballots, so equal digits keep their input order.
// Each key first lands at its tile-local sorted position in LDS (digit runs
// start at the exclusive scan of this block's histogram), then the whole tile
// is written out digit run by digit run: consecutive lanes write consecutive
// addresses of a run (an average 4096 / 256 = 16 keys) instead of 256
// scattered single keys per round.
__global__ __launch_bounds__(kBlock) void k_radix_scatter(
    const uint64_t* __restrict__ keys, const uint32_t* __restrict__ vals, int64_t n, int shift,
    const uint32_t* __restrict__ hist, const int64_t* __restrict__ offs, int64_t nblocks,
    uint64_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out) {
  __shared__ uint64_t sk[kTile];
  __shared__ uint32_t sv[kTile];
  __shared__ uint32_t wcnt[kWaves][kRadix];
  __shared__ uint32_t lstart[kRadix];
  __shared__ uint32_t lrun[kRadix];
  __shared__ int64_t gbase[kRadix];
  const int tid = threadIdx.x;
  const int wave = tid / kWave;
  const int64_t slot = static_cast<int64_t>(tid) * nblocks + blockIdx.x;
  const uint32_t cnt = hist[slot];
  gbase[tid] = offs[slot];
  lstart[tid] = cnt;
  __syncthreads();
  for (int o = 1; o < kRadix; o <<= 1) {            // inclusive scan of the block's digit counts
    const uint32_t v = tid >= o ? lstart[tid - o] : 0u;
    __syncthreads();
    lstart[tid] += v;
    __syncthreads();
  }
  const uint32_t excl = lstart[tid] - cnt;
  __syncthreads();
  lstart[tid] = excl;
  lrun[tid] = excl;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kTile;
  // all kItems keys of this thread in flight at once
  uint64_t kr[kItems];
  uint32_t vr[kItems];
#pragma unroll
  for (int r = 0; r < kItems; ++r) {
    const int64_t i = base + r * kBlock + tid;
    kr[r] = i < n ? keys[i] : 0;
    vr[r] = i < n ? (vals ? vals[i] : static_cast<uint32_t>(i)) : 0u;
  }
#pragma unroll
  for (int r = 0; r < kItems; ++r) {
#pragma unroll
    for (int w = 0; w < kWaves; ++w) wcnt[w][tid] = 0;
    __syncthreads();
    const bool valid = base + r * kBlock + tid < n;
    const uint64_t key = kr[r];
    const int d = valid ? static_cast<int>((key >> shift) & 0xFF) : 0;
    uint64_t peers = ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const bool bit = (d >> b) & 1;
      const uint64_t m = ballot(bit);
      peers &= bit ? m : ~m;
    }
    const int rank_in_wave = mbcnt(peers);
    if (valid && rank_in_wave == 0) wcnt[wave][d] = __popcll(peers);
    __syncthreads();
    if (valid) {
      uint32_t pos = lrun[d] + rank_in_wave;
      for (int w = 0; w < wave; ++w) pos += wcnt[w][d];
      sk[pos] = key;
      sv[pos] = vr[r];
    }
    __syncthreads();
    uint32_t tot = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) tot += wcnt[w][tid];
    lrun[tid] += tot;
    __syncthreads();
  }
  const int m = static_cast<int>(n - base < kTile ? n - base : kTile);
  for (int j = tid; j < m; j += kBlock) {
    const uint64_t key = sk[j];
    const int d = static_cast<int>((key >> shift) & 0xFF);
    const int64_t pos = gbase[d] + (j - static_cast<int>(lstart[d]));
    keys_out[pos] = key;
    vals_out[pos] = sv[j];
  }
}

}  // namespace

size_t radix_sort_workspace_size(int64_t n) {
  const int64_t nb = (n + kTile - 1) / kTile;
  size_t s = 0;
  s += align_up(static_cast<size_t>(n > 0 ? n : 1) * sizeof(uint64_t));  // key ping-pong
  s += align_up(static_cast<size_t>(n > 0 ? n : 1) * sizeof(uint32_t));  // val ping-pong
  s += align_up(static_cast<size_t>(kRadix * nb + 1) * sizeof(uint32_t));
  s += align_up(static_cast<size_t>(kRadix * nb + 1) * sizeof(int64_t));
  s += align_up(scan_workspace_size(kRadix * nb + 1));
  return s + 1024;
}

// Sorts keys[0..n) (and vals, identity if vals_in == nullptr) by the low
// key_bits bits; result in keys_out/vals_out.  Inputs are not modified.
hipError_t radix_sort_pairs(const uint64_t* keys_in, const uint32_t* vals_in, uint64_t* keys_out,
                            uint32_t* vals_out, int64_t n, int key_bits, void* ws,
                            size_t ws_bytes, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const int64_t nb = (n + kTile - 1) / kTile;
  Carve c(ws, ws_bytes);
  uint64_t* kt = c.take<uint64_t>(n);
  uint32_t* vt = c.take<uint32_t>(n);
  uint32_t* hist = c.take<uint32_t>(kRadix * nb + 1);
  int64_t* offs = c.take<int64_t>(kRadix * nb + 1);
  const size_t sws_bytes = scan_workspace_size(kRadix * nb + 1);
  void* sws = c.take<char>(sws_bytes);
  if (!c.ok) return hipErrorInvalidValue;
  int passes = (key_bits + 7) / 8;
  if (passes < 1) passes = 1;
  // ping-pong so the final pass lands in keys_out/vals_out
  const uint64_t* src_k = keys_in;
  const uint32_t* src_v = vals_in;
  for (int p = 0; p < passes; ++p) {
    const bool to_out = ((passes - 1 - p) % 2) == 0;
    uint64_t* dk = to_out ? keys_out : kt;
    uint32_t* dv = to_out ? vals_out : vt;
    k_radix_hist<<<static_cast<unsigned>(nb), kBlock, 0, stream>>>(src_k, n, 8 * p, hist, nb);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = scan_exclusive<uint32_t>(hist, offs, kRadix * nb, sws, sws_bytes, stream);
    if (e != hipSuccess) return e;
    k_radix_scatter<<<static_cast<unsigned>(nb), kBlock, 0, stream>>>(src_k, src_v, n, 8 * p, hist,
                                                                      offs, nb, dk, dv);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    src_k = dk;
    src_v = dv;
  }
  return hipSuccess;
}

}  // namespace dps
