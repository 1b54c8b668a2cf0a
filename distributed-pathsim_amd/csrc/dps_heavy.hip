// Venue skipping support (include/dpathsim.h, dps_venue_skip): the heavy-venue
// set and the dense table of C over it.  The hot kernel (dps_cct1.hip) stops
// scattering a heavy venue's C^T buckets once the row's k-th score makes that
// venue unable to lift a target to the top-k on its own, and completes each
// flagged target's pairwise walk M[x,y] (DPathSim_APVPA.py:90-109) from this
// table: one 64-byte row per target (n_hv = 32 uint16 counts), read only for
// the few targets that pass the lowered threshold.
#include "dps_common.hpp"

namespace dps {
namespace {

constexpr int kSelT = 1024;

// One workgroup: the smallest threshold thr >= 1 with |{v : n_v >= thr}| <=
// n_hv, i.e. one above the (n_hv + 1)-th largest n_v (1 when there are at most
// n_hv venues), found by an MSB-first radix select (four 8-bit digit passes,
// an LDS histogram each; round 6 -- a 32-step binary search over the value
// range took ~0.1 ms of config3's build); then slots in venue order for the
// venues at or above it.
__global__ __launch_bounds__(kSelT) void k_hv_select(const uint32_t* __restrict__ n_v, int64_t n_mids,
                                                     int n_hv, int32_t* __restrict__ hv_slot) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t pre[kSelT];
  __shared__ uint32_t sel[2];            // digit, count above it
  const int tid = threadIdx.x;
  uint64_t thr = 1;
  if (n_mids > n_hv) {
    uint32_t prefix = 0, mask = 0, want = static_cast<uint32_t>(n_hv) + 1u;   // rank, descending
    for (int shift = 24; shift >= 0; shift -= 8) {
      if (tid < 256) hist[tid] = 0;
      __syncthreads();
      for (int64_t i = tid; i < n_mids; i += kSelT) {
        const uint32_t v = n_v[i];
        if ((v & mask) == prefix) atomicAdd(&hist[(v >> shift) & 255u], 1u);
      }
      __syncthreads();
      if (tid < kWave) {
        // lane l holds bins 4l..4l+3; above = the count in the bins past them
        uint32_t h[4], own = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) { h[j] = hist[4 * tid + j]; own += h[j]; }
        const uint32_t incl = wave_inclusive_sum(own);
        const uint32_t total = __shfl(incl, kWave - 1, kWave);
        uint32_t above = total - incl;
        if (above < want && want <= above + own) {
#pragma unroll
          for (int j = 3; j >= 0; --j) {
            if (above < want && want <= above + h[j]) { sel[0] = 4u * tid + j; sel[1] = above; }
            above += h[j];
          }
        }
      }
      __syncthreads();
      prefix |= sel[0] << shift;
      mask |= 255u << shift;
      want -= sel[1];
      __syncthreads();                   // sel / hist reused by the next pass
    }
    thr = static_cast<uint64_t>(prefix) + 1u;
  }
  // contiguous venue ranges per thread, exclusive scan of their heavy counts
  const int64_t per = (n_mids + kSelT - 1) / kSelT;
  const int64_t b = tid * per, e = b + per < n_mids ? b + per : n_mids;
  uint32_t own = 0;
  for (int64_t i = b; i < e; ++i) own += static_cast<uint64_t>(n_v[i]) >= thr;
  pre[tid] = own;
  __syncthreads();
  for (int d = 1; d < kSelT; d <<= 1) {
    const uint32_t t = tid >= d ? pre[tid - d] : 0u;
    __syncthreads();
    pre[tid] += t;
    __syncthreads();
  }
  int slot = static_cast<int>(pre[tid] - own);
  for (int64_t i = b; i < e; ++i)
    hv_slot[i] = static_cast<uint64_t>(n_v[i]) >= thr ? slot++ : -1;
}

// hv_c[label(y) * n_hv + hv_slot[v]] = C[y,v]: 16 lanes per author row.
__global__ __launch_bounds__(256) void k_hv_table(const int64_t* __restrict__ c_ptr,
                                                  const int32_t* __restrict__ c_col,
                                                  const int32_t* __restrict__ c_val,
                                                  const int32_t* __restrict__ t_rank,
                                                  int64_t n_targets,
                                                  const int32_t* __restrict__ hv_slot, int n_hv,
                                                  uint16_t* __restrict__ hv_c) {
  const int sub = threadIdx.x & 15;
  for (int64_t y = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) >> 4; y < n_targets;
       y += (static_cast<int64_t>(gridDim.x) * 256) >> 4) {
    const int64_t lab = t_rank ? t_rank[y] : y;
    const int64_t b = c_ptr[y], e = c_ptr[y + 1];
    for (int64_t j = b + sub; j < e; j += 16) {
      const int sl = hv_slot[c_col[j]];
      if (sl >= 0) {
        const int cv = c_val[j];
        hv_c[lab * n_hv + sl] = static_cast<uint16_t>(cv < 0xFFFF ? cv : 0xFFFF);
      }
    }
  }
}

}  // namespace
}  // namespace dps

using namespace dps;

extern "C" {

int dps_heavy_venues(const uint32_t* n_v, int64_t n_mids, int32_t n_hv, int32_t* hv_slot,
                     void* stream) {
  DPS_REQUIRE(n_hv >= 1 && n_hv <= 64, DPS_ERR_INVALID, "n_hv must be in [1, 64], got %d", n_hv);
  DPS_REQUIRE(n_mids >= 0 && n_mids < INT32_MAX, DPS_ERR_INVALID, "bad n_mids");
  if (n_mids == 0) return DPS_OK;
  DPS_REQUIRE(n_v && hv_slot, DPS_ERR_INVALID, "null n_v / hv_slot");
  auto st = static_cast<hipStream_t>(stream);
  k_hv_select<<<1, kSelT, 0, st>>>(n_v, n_mids, n_hv, hv_slot);
  DPS_LAUNCHED();
  return DPS_OK;
}

int dps_heavy_table(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                    const int32_t* t_rank, int64_t n_targets, const int32_t* hv_slot, int32_t n_hv,
                    uint16_t* hv_c, void* stream) {
  DPS_REQUIRE(n_hv >= 1 && n_hv <= 64, DPS_ERR_INVALID, "n_hv must be in [1, 64], got %d", n_hv);
  DPS_REQUIRE(n_targets >= 0 && n_targets < INT32_MAX, DPS_ERR_INVALID, "bad n_targets");
  if (n_targets == 0) return DPS_OK;
  DPS_REQUIRE(c_ptr && c_col && c_val && hv_slot && hv_c, DPS_ERR_INVALID, "null array");
  auto st = static_cast<hipStream_t>(stream);
  DPS_HIP_RET(hipMemsetAsync(hv_c, 0, static_cast<size_t>(n_targets) * n_hv * sizeof(uint16_t), st));
  k_hv_table<<<grid_for(n_targets * 16, 256), 256, 0, st>>>(c_ptr, c_col, c_val, t_rank, n_targets,
                                                            hv_slot, n_hv, hv_c);
  DPS_LAUNCHED();
  return DPS_OK;
}

}  // extern "C"
