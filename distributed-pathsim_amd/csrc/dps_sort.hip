// Stable LSD radix sort of (uint64 key, uint32 value) pairs, 8- or 9-bit digits.
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
constexpr int kMaxDigit = 9;            // digit widths 8..9 bits (round 5: 18-bit keys in 2 passes)
constexpr int kMaxRadix = 1 << kMaxDigit;

// Digit of a key in the pass at `shift`, `bits` wide (the last pass may be
// narrower than D: bits above the caller's key_bits never take part).
__device__ __forceinline__ int digit_of(uint64_t key, int shift, uint32_t mask) {
  return static_cast<int>((key >> shift) & mask);
}

template <int D>
__global__ __launch_bounds__(kBlock) void k_radix_hist(const uint64_t* __restrict__ keys,
                                                       int64_t n, int shift, uint32_t mask,
                                                       uint32_t* __restrict__ hist,
                                                       int64_t nblocks) {
  constexpr int R = 1 << D;
  __shared__ uint32_t h[R];
  for (int d = threadIdx.x; d < R; d += kBlock) h[d] = 0;
  __syncthreads();
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kTile;
#pragma unroll 4
  for (int r = 0; r < kItems; ++r) {
    const int64_t i = base + r * kBlock + threadIdx.x;
    if (i < n) atomicAdd(&h[digit_of(keys[i], shift, mask)], 1u);
  }
  __syncthreads();
  for (int d = threadIdx.x; d < R; d += kBlock)
    hist[static_cast<int64_t>(d) * nblocks + blockIdx.x] = h[d];
}

// Stable scatter, staged through LDS: the tile is consumed in kItems rounds
// of 256 keys in index order; inside a round keys are ranked by (wave, lane)
// with per-wave multi-split ballots (one per digit bit), so equal digits keep
// their input order.  Each key first lands at its tile-local sorted position
// in LDS (digit runs start at the exclusive scan of this block's histogram),
// then the whole tile is written out digit run by digit run: consecutive lanes
// write consecutive addresses of a run instead of 256 scattered single keys
// per round.  Thread t owns digits t*P .. t*P+P-1 (P = R / 256).
template <int D>
__global__ __launch_bounds__(kBlock) void k_radix_scatter(
    const uint64_t* __restrict__ keys, const uint32_t* __restrict__ vals, int64_t n, int shift,
    uint32_t mask, const uint32_t* __restrict__ hist, const int64_t* __restrict__ offs,
    int64_t nblocks, uint64_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out) {
  constexpr int R = 1 << D;
  constexpr int P = R / kBlock;
  static_assert(P >= 1 && P * kBlock == R, "digit width 8..9");
  __shared__ uint64_t sk[kTile];
  __shared__ uint32_t sv[kTile];
  __shared__ uint32_t wcnt[kWaves][R];
  __shared__ uint32_t lstart[R];
  __shared__ uint32_t lrun[R];
  __shared__ int64_t gbase[R];
  __shared__ uint32_t tsum[kBlock];
  const int tid = threadIdx.x;
  const int wave = tid / kWave;
  uint32_t cnt[P];
  uint32_t mine = 0;
#pragma unroll
  for (int q = 0; q < P; ++q) {
    const int d = tid * P + q;
    const int64_t slot = static_cast<int64_t>(d) * nblocks + blockIdx.x;
    cnt[q] = hist[slot];
    gbase[d] = offs[slot];
    mine += cnt[q];
  }
  tsum[tid] = mine;
  __syncthreads();
  for (int o = 1; o < kBlock; o <<= 1) {            // inclusive scan of the threads' digit counts
    const uint32_t v = tid >= o ? tsum[tid - o] : 0u;
    __syncthreads();
    tsum[tid] += v;
    __syncthreads();
  }
  uint32_t run = tsum[tid] - mine;
#pragma unroll
  for (int q = 0; q < P; ++q) {
    const int d = tid * P + q;
    lstart[d] = run;
    lrun[d] = run;
    run += cnt[q];
  }
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
    for (int w = 0; w < kWaves; ++w)
#pragma unroll
      for (int q = 0; q < P; ++q) wcnt[w][tid * P + q] = 0;
    __syncthreads();
    const bool valid = base + r * kBlock + tid < n;
    const uint64_t key = kr[r];
    const int d = valid ? digit_of(key, shift, mask) : 0;
    uint64_t peers = ballot(valid);
#pragma unroll
    for (int b = 0; b < D; ++b) {
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
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const int dd = tid * P + q;
      uint32_t tot = 0;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) tot += wcnt[w][dd];
      lrun[dd] += tot;
    }
    __syncthreads();
  }
  const int m = static_cast<int>(n - base < kTile ? n - base : kTile);
  for (int j = tid; j < m; j += kBlock) {
    const uint64_t key = sk[j];
    const int d = digit_of(key, shift, mask);
    const int64_t pos = gbase[d] + (j - static_cast<int>(lstart[d]));
    keys_out[pos] = key;
    vals_out[pos] = sv[j];
  }
}

template <int D>
hipError_t radix_pass(const uint64_t* src_k, const uint32_t* src_v, int64_t n, int shift, int bits,
                      uint32_t* hist, int64_t* offs, void* sws, size_t sws_bytes, int64_t nb,
                      uint64_t* dk, uint32_t* dv, hipStream_t stream) {
  const uint32_t mask = (1u << bits) - 1u;
  k_radix_hist<D><<<static_cast<unsigned>(nb), kBlock, 0, stream>>>(src_k, n, shift, mask, hist, nb);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = scan_exclusive<uint32_t>(hist, offs, (int64_t(1) << D) * nb, sws, sws_bytes, stream);
  if (e != hipSuccess) return e;
  k_radix_scatter<D><<<static_cast<unsigned>(nb), kBlock, 0, stream>>>(src_k, src_v, n, shift, mask,
                                                                       hist, offs, nb, dk, dv);
  return hipGetLastError();
}

}  // namespace

size_t radix_sort_workspace_size(int64_t n) {
  const int64_t nb = (n + kTile - 1) / kTile;
  size_t s = 0;
  s += align_up(static_cast<size_t>(n > 0 ? n : 1) * sizeof(uint64_t));  // key ping-pong
  s += align_up(static_cast<size_t>(n > 0 ? n : 1) * sizeof(uint32_t));  // val ping-pong
  s += align_up(static_cast<size_t>(kMaxRadix * nb + 1) * sizeof(uint32_t));
  s += align_up(static_cast<size_t>(kMaxRadix * nb + 1) * sizeof(int64_t));
  s += align_up(scan_workspace_size(kMaxRadix * nb + 1));
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
  uint32_t* hist = c.take<uint32_t>(kMaxRadix * nb + 1);
  int64_t* offs = c.take<int64_t>(kMaxRadix * nb + 1);
  const size_t sws_bytes = scan_workspace_size(kMaxRadix * nb + 1);
  void* sws = c.take<char>(sws_bytes);
  if (!c.ok) return hipErrorInvalidValue;
  // fewest passes of 8..9-bit digits (round 5; 8-bit digits only before):
  // 18-bit keys (config4's mids) take 2 passes instead of 3
  const int kb = key_bits < 1 ? 1 : key_bits;
  int passes = (kb + kMaxDigit - 1) / kMaxDigit;
  int dbits = (kb + passes - 1) / passes;
  if (dbits < 8) dbits = 8;
  // ping-pong so the final pass lands in keys_out/vals_out
  const uint64_t* src_k = keys_in;
  const uint32_t* src_v = vals_in;
  for (int p = 0; p < passes; ++p) {
    const bool to_out = ((passes - 1 - p) % 2) == 0;
    uint64_t* dk = to_out ? keys_out : kt;
    uint32_t* dv = to_out ? vals_out : vt;
    const int shift = dbits * p;
    const int bits = kb - shift < dbits ? kb - shift : dbits;   // >= 1
    hipError_t e;
    if (dbits == 8)
      e = radix_pass<8>(src_k, src_v, n, shift, bits, hist, offs, sws, sws_bytes, nb, dk, dv, stream);
    else
      e = radix_pass<9>(src_k, src_v, n, shift, bits, hist, offs, sws, sws_bytes, nb, dk, dv, stream);
    if (e != hipSuccess) return e;
    src_k = dk;
    src_v = dv;
  }
  return hipSuccess;
}

}  // namespace dps
