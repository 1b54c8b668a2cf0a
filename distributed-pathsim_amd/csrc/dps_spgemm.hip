// A3: C = W_AP . W_PX as a wavefront-cooperative hash SpGEMM (SURVEY.md §8a
// row A3; the join A->P->V of the motif, DPathSim_APVPA.py:72-74).
//
// C[a,v] = |{p : (a,p) in AP, (p,v) in PX}| for every output row a, columns
// ascending.  Two passes over the inputs, no expanded intermediate array:
//   symbolic  u[a] = number of distinct venues of row a; scan -> c_ptr;
//   numeric   the same per-row work again, writing (v, count) at c_ptr[a].
// Per row the expansion length L = sum_{p in AP[a]} |PX[p]| picks the path:
//   L <= 16         one LANE: the venues are gathered into a per-lane LDS
//                   slot, loaded into 16 registers and sorted by a bitonic
//                   network; runs give the counts (the common case: APVPA
//                   authors write a handful of papers, one venue each);
//   16 < L <= 64    one WAVE: one expanded venue per lane, wave bitonic sort,
//                   heads and run lengths by ballot;
//   64 < L <= 4096  one WORKGROUP (deferred to a list): LDS hash table of
//                   8192 slots (open addressing, atomicCAS inserts recording
//                   the occupied slots, atomicAdd counts); numeric sorts the
//                   occupied slots by venue with an LDS bitonic network;
//   L > 4096        one workgroup with a global scratch region of max_expand
//                   slots: the venues are sorted there in place (bitonic),
//                   then unique + run lengths.
// Both passes are enqueue-only (no host read-back); the long-row list count
// lives in the workspace.
#include "dps_common.hpp"

namespace dps {
namespace {

constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kLaneCap = 16;        // expansion a lane sorts in registers
constexpr int kHashSlots = 8192;    // LDS hash slots of the workgroup path
constexpr int kHashCap = 4096;      // expansion the LDS hash takes (load <= 1/2)
constexpr int kHugeBlocks = 32;     // workgroups (and scratch regions) of the L > 4096 path
constexpr int kRankSortMax = 1024;  // distinct keys of a row sorted by ranking (numeric pass)

__device__ __forceinline__ int64_t out_row(const int32_t* rows, int64_t i) {
  return rows ? static_cast<int64_t>(rows[i]) : i;
}

// Expansion of one row into a lane's LDS slot: returns L (counting stops past
// `stop`), the first min(L, kLaneCap) venues stored.  Papers are taken four
// at a time so the dependent loads (paper -> venue range -> venue) of four
// papers are in flight together.
__device__ __forceinline__ int64_t lane_gather(int32_t* __restrict__ slot,
                                               const int32_t* __restrict__ ap_col,
                                               const int64_t* __restrict__ px_ptr,
                                               const int32_t* __restrict__ px_col, int64_t b,
                                               int64_t e, int64_t stop) {
  int64_t n = 0;
  for (int64_t j = b; j < e && n <= stop; j += 4) {
    int32_t p[4];
    int64_t pb[4], pe[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) p[u] = j + u < e ? ap_col[j + u] : -1;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      pb[u] = p[u] >= 0 ? px_ptr[p[u]] : 0;
      pe[u] = p[u] >= 0 ? px_ptr[p[u] + 1] : 0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      for (int64_t q = pb[u]; q < pe[u]; ++q) {
        if (n < kLaneCap) slot[n] = px_col[q];
        ++n;
      }
  }
  return n;
}

// Lane path: the row's (<= 16) venues (already in the slot) sorted in
// registers; returns the number of distinct venues and, when col != nullptr,
// writes (v, count) ascending.
__device__ __forceinline__ int lane_row(const int32_t* __restrict__ slot, int n,
                                        int32_t* __restrict__ col, int32_t* __restrict__ val) {
  int32_t v[kLaneCap];
#pragma unroll
  for (int i = 0; i < kLaneCap; ++i) v[i] = i < n ? slot[i] : INT_MAX;
#pragma unroll
  for (int k = 2; k <= kLaneCap; k <<= 1) {
#pragma unroll
    for (int jj = k >> 1; jj > 0; jj >>= 1) {
#pragma unroll
      for (int i = 0; i < kLaneCap; ++i) {
        const int l = i ^ jj;
        if (l > i) {
          const int32_t a = v[i], c = v[l];
          const bool up = (i & k) == 0;
          v[i] = up ? min(a, c) : max(a, c);
          v[l] = up ? max(a, c) : min(a, c);
        }
      }
    }
  }
  int u = 0, run = 0;
#pragma unroll
  for (int i = 0; i < kLaneCap; ++i) {
    if (i < n) {
      if (i == 0 || v[i] != v[i - 1]) {
        if (col && u > 0) val[u - 1] = run;
        if (col) col[u] = v[i];
        ++u;
        run = 1;
      } else {
        ++run;
      }
    }
  }
  if (col && u > 0) val[u - 1] = run;
  return u;
}

// ---- pass 1 / pass 2: lane tier (L <= 16) and wave tier (16 < L <= 64) --------
// numeric == false: u[i] = distinct venues; rows with L > 64 get u[i] = 0 and
// are appended to long_list.  numeric == true: rows with L <= 64 write their
// (v, count) at c_ptr[i]; long rows are left to k_hash_long.
template <bool kNumeric>
__global__ __launch_bounds__(kBlock) void k_hash_rows(
    const int64_t* __restrict__ ap_ptr, const int32_t* __restrict__ ap_col,
    const int32_t* __restrict__ rows, int64_t n_out, const int64_t* __restrict__ px_ptr,
    const int32_t* __restrict__ px_col, uint32_t* __restrict__ u, int32_t* __restrict__ long_list,
    unsigned* __restrict__ n_long, const int64_t* __restrict__ c_ptr, int32_t* __restrict__ c_col,
    int32_t* __restrict__ c_val) {
  __shared__ int32_t scratch[kBlock * kLaneCap];
  int32_t* slot = scratch + threadIdx.x * kLaneCap;
  const int lane = lane_id();
  const int64_t wave0 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWavesPerBlock;
  for (int64_t i0 = wave0 * kWave; i0 < n_out; i0 += nwaves * kWave) {   // wave-uniform
    const int64_t i = i0 + lane;
    int64_t b = 0, e = 0, L = 0;
    if (i < n_out) {
      const int64_t r = out_row(rows, i);
      b = ap_ptr[r];
      e = ap_ptr[r + 1];
      L = lane_gather(slot, ap_col, px_ptr, px_col, b, e, kWave);
      if (L <= kLaneCap) {
        if (kNumeric) {
          const int64_t o = c_ptr[i];
          lane_row(slot, static_cast<int>(L), c_col + o, c_val + o);
        } else {
          u[i] = static_cast<uint32_t>(lane_row(slot, static_cast<int>(L), nullptr, nullptr));
        }
      } else if (L > kWave && !kNumeric) {
        u[i] = 0;
        long_list[atomicAdd(n_long, 1u)] = static_cast<int32_t>(i);
      }
    }
    // wave tier: one row at a time, one expanded venue per lane, bitonic sort
    uint64_t todo = ballot(L > kLaneCap && L <= kWave);
    while (todo) {
      const int src = __ffsll(static_cast<long long>(todo)) - 1;
      todo &= todo - 1;
      const int64_t bb = readlane(b, src), ee = readlane(e, src);
      // gather the (<= 64) expanded venues through LDS (the wave's lane slots):
      // 64 papers at a time, a wave prefix over their venue counts
      int32_t* ws = scratch + (threadIdx.x / kWave) * kWave * kLaneCap;
      int len = 0;
      for (int64_t c0 = bb; c0 < ee; c0 += kWave) {
        int64_t pb = 0;
        int pl = 0;
        if (c0 + lane < ee) {
          const int32_t p = ap_col[c0 + lane];
          pb = px_ptr[p];
          pl = static_cast<int>(px_ptr[p + 1] - pb);
        }
        const int inc = wave_inclusive_sum(pl);
        for (int t = 0; t < pl; ++t) ws[len + inc - pl + t] = px_col[pb + t];
        len += readlane(inc, kWave - 1);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      int v = lane < len ? ws[lane] : INT_MAX;
      __builtin_amdgcn_wave_barrier();
      v = wave_bitonic_sort(v);
      const int prev = __shfl_up(v, 1, kWave);
      const bool first = lane < len && (lane == 0 || v != prev);
      const uint64_t mask = ballot(first);
      const int64_t i_row = i0 + src;
      if (kNumeric) {
        if (first) {
          const uint64_t above = mask & ~((2ull << lane) - 1ull);
          const int next = above ? (__ffsll(static_cast<long long>(above)) - 1) : len;
          const int64_t o = c_ptr[i_row] + mbcnt(mask);
          c_col[o] = v;
          c_val[o] = next - lane;
        }
      } else if (lane == 0) {
        u[i_row] = static_cast<uint32_t>(__popcll(mask));
      }
    }
  }
}

// ---- long rows: one workgroup per row -----------------------------------------
__device__ __forceinline__ uint32_t hash_slot(uint32_t v) {
  return (v * 2654435761u) >> (32 - 13);   // 8192 slots
}

__device__ int block_sum(int v, int* lds_w) {
  const int lane = lane_id(), wave = threadIdx.x / kWave;
  v = wave_sum(v);
  if (lane == 0) lds_w[wave] = v;
  __syncthreads();
  int t = 0;
#pragma unroll
  for (int w = 0; w < kWavesPerBlock; ++w) t += lds_w[w];
  __syncthreads();
  return t;
}

// Exclusive rank of `flag` over the block (+ total).
__device__ int block_rank(bool flag, int* lds_w, int* total) {
  const int lane = lane_id(), wave = threadIdx.x / kWave;
  const uint64_t m = ballot(flag);
  if (lane == 0) lds_w[wave] = __popcll(m);
  __syncthreads();
  int off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kWavesPerBlock; ++w) {
    if (w < wave) off += lds_w[w];
    tot += lds_w[w];
  }
  __syncthreads();
  *total = tot;
  return off + mbcnt(m);
}

// Ascending bitonic sort of n (key, val) pairs in LDS or global memory with
// virtual +inf padding to a power of two (minimum to the lower index).
template <class KP, class VP>
__device__ void block_sort_pairs(KP key, VP val, int n) {
  int n2 = 1;
  while (n2 < n) n2 <<= 1;
  for (int k = 2; k <= n2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = threadIdx.x; t < n2 / 2; t += kBlock) {
        const int lo = (j == (k >> 1)) ? (t / j) * k + (t % j) : (t / j) * 2 * j + (t % j);
        const int hi = (j == (k >> 1)) ? (t / j) * k + k - 1 - (t % j) : lo + j;
        if (hi < n) {
          const int32_t a = key[lo], b = key[hi];
          if (b < a) {
            key[lo] = b; key[hi] = a;
            if (val) { const int32_t x = val[lo]; val[lo] = val[hi]; val[hi] = x; }
          }
        }
      }
      __syncthreads();
    }
  }
}

template <bool kNumeric>
__global__ __launch_bounds__(kBlock) void k_hash_long(
    const int64_t* __restrict__ ap_ptr, const int32_t* __restrict__ ap_col,
    const int32_t* __restrict__ rows, const int64_t* __restrict__ px_ptr,
    const int32_t* __restrict__ px_col, uint32_t* __restrict__ u,
    const int32_t* __restrict__ long_list, const unsigned* __restrict__ n_long,
    const int64_t* __restrict__ c_ptr, int32_t* __restrict__ c_col, int32_t* __restrict__ c_val,
    int32_t* __restrict__ huge_scratch, int64_t max_expand, int32_t* __restrict__ status) {
  __shared__ int32_t hkey[kHashSlots];
  __shared__ int32_t hcnt[kHashSlots];
  __shared__ int32_t occ[kHashCap];          // occupied slots of the current row
  __shared__ int n_occ;
  __shared__ int lds_w[kWavesPerBlock];
  __shared__ int64_t lds_off[kWavesPerBlock];
  const int lane = lane_id(), wave = threadIdx.x / kWave;
  const unsigned nl = *n_long;
  for (int s = threadIdx.x; s < kHashSlots; s += kBlock) { hkey[s] = -1; hcnt[s] = 0; }
  if (threadIdx.x == 0) n_occ = 0;
  __syncthreads();
  for (unsigned li = blockIdx.x; li < nl; li += gridDim.x) {
    const int64_t i = long_list[li];
    const int64_t r = out_row(rows, i);
    const int64_t b = ap_ptr[r], e = ap_ptr[r + 1];
    // expansion length (block-cooperative)
    int64_t Lp = 0;
    for (int64_t j = b + threadIdx.x; j < e; j += kBlock) {
      const int32_t p = ap_col[j];
      Lp += px_ptr[p + 1] - px_ptr[p];
    }
    const int64_t L = block_sum(static_cast<int>(Lp), lds_w);
    if (L <= kHashCap) {
      // insert every (paper, venue) of the row: a wave walks 64 papers at a
      // time; a successful insert records its slot in the occupied list
      for (int64_t j0 = b + wave * kWave; j0 < e; j0 += kBlock) {
        const int64_t j = j0 + lane;
        if (j < e) {
          const int32_t p = ap_col[j];
          for (int64_t q = px_ptr[p]; q < px_ptr[p + 1]; ++q) {
            const int32_t v = px_col[q];
            uint32_t h = hash_slot(static_cast<uint32_t>(v));
            for (;;) {
              const int32_t old = atomicCAS(&hkey[h], -1, v);
              if (old == -1) { occ[atomicAdd(&n_occ, 1)] = static_cast<int32_t>(h); break; }
              if (old == v) break;
              h = (h + 1) & (kHashSlots - 1);
            }
            if (kNumeric) atomicAdd(&hcnt[h], 1);
          }
        }
      }
      __syncthreads();
      const int nu = n_occ;
      if (!kNumeric) {
        if (threadIdx.x == 0) u[i] = static_cast<uint32_t>(nu);
      } else if (nu <= kRankSortMax) {
        // rank sort of the (distinct) keys: every occupied slot's position is
        // the number of smaller keys -- two barriers instead of log^2 phases
        int32_t key[kRankSortMax / kBlock], cnt[kRankSortMax / kBlock];
#pragma unroll
        for (int q = 0; q < kRankSortMax / kBlock; ++q) {
          const int t = threadIdx.x + q * kBlock;
          key[q] = t < nu ? hkey[occ[t]] : INT_MAX;
          cnt[q] = t < nu ? hcnt[occ[t]] : 0;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kRankSortMax / kBlock; ++q) {
          const int t = threadIdx.x + q * kBlock;
          if (t < nu) occ[t] = key[q];                 // occ now holds the keys
        }
        __syncthreads();
        const int64_t o = c_ptr[i];
#pragma unroll
        for (int q = 0; q < kRankSortMax / kBlock; ++q) {
          const int t = threadIdx.x + q * kBlock;
          if (t >= nu) continue;
          int r = 0;
          for (int w = 0; w < nu; ++w) r += occ[w] < key[q] ? 1 : 0;
          c_col[o + r] = key[q];
          c_val[o + r] = cnt[q];
        }
        __syncthreads();
        // restore the slot list for the reset below
        for (int t = threadIdx.x; t < nu; t += kBlock) {
          uint32_t h = hash_slot(static_cast<uint32_t>(occ[t]));
          while (hkey[h] != occ[t]) h = (h + 1) & (kHashSlots - 1);
          occ[t] = static_cast<int32_t>(h);
        }
      } else {
        // sort the occupied slots by their key, then write (key, count)
        int n2 = 1;
        while (n2 < nu) n2 <<= 1;
        for (int k = 2; k <= n2; k <<= 1) {
          for (int jd = k >> 1; jd > 0; jd >>= 1) {
            for (int t = threadIdx.x; t < n2 / 2; t += kBlock) {
              const int lo = (jd == (k >> 1)) ? (t / jd) * k + (t % jd) : (t / jd) * 2 * jd + (t % jd);
              const int hi = (jd == (k >> 1)) ? (t / jd) * k + k - 1 - (t % jd) : lo + jd;
              if (hi < nu) {
                const int32_t sa = occ[lo], sb = occ[hi];
                if (hkey[sb] < hkey[sa]) { occ[lo] = sb; occ[hi] = sa; }
              }
            }
            __syncthreads();
          }
        }
        const int64_t o = c_ptr[i];
        for (int t = threadIdx.x; t < nu; t += kBlock) {
          c_col[o + t] = hkey[occ[t]];
          c_val[o + t] = hcnt[occ[t]];
        }
      }
      __syncthreads();
      for (int t = threadIdx.x; t < nu; t += kBlock) { hkey[occ[t]] = -1; hcnt[occ[t]] = 0; }
      if (threadIdx.x == 0) n_occ = 0;
      __syncthreads();
      continue;
    }
    // L > 4096: left to the first kHugeBlocks blocks, which own the global
    // scratch regions (second loop below)
  }
  // huge rows: the first kHugeBlocks blocks re-walk the list and take them
  if (blockIdx.x >= kHugeBlocks) return;
  int32_t* scr = huge_scratch + static_cast<int64_t>(blockIdx.x) * max_expand;
  for (unsigned li = blockIdx.x; li < nl; li += kHugeBlocks) {
    const int64_t i = long_list[li];
    const int64_t r = out_row(rows, i);
    const int64_t b = ap_ptr[r], e = ap_ptr[r + 1];
    int64_t Lp = 0;
    for (int64_t j = b + threadIdx.x; j < e; j += kBlock) {
      const int32_t p = ap_col[j];
      Lp += px_ptr[p + 1] - px_ptr[p];
    }
    const int64_t L = block_sum(static_cast<int>(Lp), lds_w);
    if (L <= kHashCap) continue;
    if (L > max_expand) {   // the caller's bound was wrong: flag it, leave the row
      if (threadIdx.x == 0 && status) *status = DPS_ERR_OVERFLOW;
      continue;
    }
    // expand into scratch: each wave takes 64 papers at a time, offsets by scan
    int64_t base = 0;
    for (int64_t j0 = b; j0 < e; j0 += kBlock) {
      const int64_t j = j0 + threadIdx.x;
      int64_t pb = 0, pl = 0;
      if (j < e) {
        const int32_t p = ap_col[j];
        pb = px_ptr[p];
        pl = px_ptr[p + 1] - pb;
      }
      const int64_t inc = wave_inclusive_sum(pl);
      if (lane == kWave - 1) lds_off[wave] = inc;
      __syncthreads();
      int64_t off = base, tot = 0;
#pragma unroll
      for (int w = 0; w < kWavesPerBlock; ++w) {
        if (w < wave) off += lds_off[w];
        tot += lds_off[w];
      }
      __syncthreads();
      const int64_t o = off + inc - pl;
      for (int64_t t = 0; t < pl; ++t) scr[o + t] = px_col[pb + t];
      base += tot;
    }
    __syncthreads();
    block_sort_pairs(scr, static_cast<int32_t*>(nullptr), static_cast<int>(L));
    // unique + counts: a head is where the value changes
    int nu = 0, total = 0;
    const int64_t o = kNumeric ? c_ptr[i] : 0;
    for (int64_t t0 = 0; t0 < L; t0 += kBlock) {
      const int64_t t = t0 + threadIdx.x;
      const bool head = t < L && (t == 0 || scr[t] != scr[t - 1]);
      const int pos = block_rank(head, lds_w, &total);
      if (kNumeric && head) {
        int64_t nx = t + 1;
        while (nx < L && scr[nx] == scr[t]) ++nx;
        c_col[o + nu + pos] = scr[t];
        c_val[o + nu + pos] = static_cast<int32_t>(nx - t);
      }
      nu += total;
    }
    if (!kNumeric && threadIdx.x == 0) u[i] = static_cast<uint32_t>(nu);
    __syncthreads();
  }
}

__global__ void k_total(const int64_t* c_ptr, int64_t n, int64_t* nnz) { *nnz = c_ptr[n]; }

// ---- single-mid path: every paper has at most one mid ----------------------
// The expansion of row a is then exactly its AP segment with every paper
// replaced by its mid (or by INT_MAX when it has none): a segmented sort +
// unique over the AP segments (seg_unique) whose loads gather vp[ap_col[j]]
// gives the distinct mids and their counts.
// mid of every paper (INT_MAX: none), coalesced over the PX rows, so the
// per-entry gather in the segmented sort's loads is one random 4-byte read
// instead of three dependent ones
__global__ __launch_bounds__(kBlock) void k_paper_mid(const int64_t* __restrict__ px_ptr,
                                                      const int32_t* __restrict__ px_col,
                                                      int64_t n_papers, int32_t* __restrict__ vp) {
  for (int64_t p = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; p < n_papers;
       p += static_cast<int64_t>(gridDim.x) * kBlock) {
    const int64_t q = px_ptr[p];
    vp[p] = px_ptr[p + 1] > q ? px_col[q] : INT_MAX;
  }
}

// Paper -> mid map straight from the typed PX pairs (no PX CSR): with at most
// one raw PX edge per paper (the single-mid case, decided on the host) the
// pairs are already distinct and every paper is written at most once.
__global__ __launch_bounds__(kBlock) void k_paper_mid_pairs(const int32_t* __restrict__ px_paper,
                                                            const int32_t* __restrict__ px_mid,
                                                            int64_t cap, const int64_t* n_dev,
                                                            int32_t* __restrict__ vp) {
  const int64_t n = n_dev ? min(*n_dev, cap) : cap;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * kBlock)
    vp[px_paper[i]] = px_mid[i];
}

__global__ __launch_bounds__(kBlock) void k_fill_i32(int32_t* __restrict__ a, int64_t n, int32_t v) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * kBlock)
    a[i] = v;
}

// After the segmented unique: drop a trailing INT_MAX head (papers without a
// mid) from each row's count.
__global__ __launch_bounds__(kBlock) void k_drop_none(const int32_t* __restrict__ mids,
                                                      const int64_t* __restrict__ seg_ptr,
                                                      int64_t n_seg, int64_t* __restrict__ uniq) {
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; r < n_seg;
       r += static_cast<int64_t>(gridDim.x) * kBlock) {
    const int64_t nu = uniq[r];
    if (nu > 0 && mids[seg_ptr[r] + nu - 1] == INT_MAX) uniq[r] = nu - 1;
  }
}

// Compact the segment heads into C (single-mid path).
__global__ __launch_bounds__(kBlock) void k_compact_mids(const int32_t* __restrict__ mids,
                                                         const int32_t* __restrict__ cnt,
                                                         const int64_t* __restrict__ seg_ptr,
                                                         const int64_t* __restrict__ c_ptr,
                                                         int64_t n_seg, int32_t* __restrict__ col,
                                                         int32_t* __restrict__ val) {
  const int64_t wave0 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWavesPerBlock;
  for (int64_t s0 = wave0 * kWave; s0 < n_seg; s0 += nwaves * kWave)
    compact_heads_wave(mids, cnt, seg_ptr, c_ptr, n_seg, col, val, s0);
}

}  // namespace
}  // namespace dps

using namespace dps;

extern "C" {

size_t dps_spgemm_hash_workspace_size(int64_t n_out_rows, int64_t max_row_expand) {
  const size_t n = static_cast<size_t>(n_out_rows > 0 ? n_out_rows : 1);
  const size_t hm = max_row_expand > kHashCap ? static_cast<size_t>(max_row_expand) : 1;
  size_t s = 0;
  s += align_up(n * sizeof(uint32_t));          // u
  s += align_up(n * sizeof(int32_t));           // long_list
  s += align_up(sizeof(unsigned) * 4);          // n_long
  s += align_up(scan_workspace_size(n_out_rows + 1));
  s += align_up(kHugeBlocks * hm * sizeof(int32_t));   // huge-row scratch
  return s + 1024;
}

size_t dps_spgemm_single_workspace_size(int64_t n_out_rows, int64_t nnz_ap, int64_t n_papers) {
  const size_t n = static_cast<size_t>(n_out_rows > 0 ? n_out_rows : 1);
  const size_t e = static_cast<size_t>(nnz_ap > 0 ? nnz_ap : 1);
  size_t s = 0;
  s += align_up(static_cast<size_t>(n_papers > 0 ? n_papers : 1) * sizeof(int32_t));   // vp
  s += align_up(e * sizeof(int32_t));           // mids of the AP entries
  s += align_up(e * sizeof(int32_t));           // run counts
  s += align_up(n * sizeof(int64_t));           // uniq
  s += align_up(scan_workspace_size(n_out_rows + 1));
  s += align_up(seg_unique_workspace_size(n_out_rows));
  return s + 1024;
}

int dps_paper_mid_map(const int32_t* px_paper, const int32_t* px_mid, int64_t n_px_cap,
                      const int64_t* n_px_dev, int64_t n_papers, int32_t* vp, void* stream) {
  DPS_REQUIRE(n_px_cap >= 0 && n_papers >= 0, DPS_ERR_INVALID, "negative size");
  DPS_REQUIRE(n_papers == 0 || vp, DPS_ERR_INVALID, "null vp");
  auto st = static_cast<hipStream_t>(stream);
  if (n_papers == 0) return DPS_OK;
  k_fill_i32<<<grid_for(n_papers, kBlock), kBlock, 0, st>>>(vp, n_papers, INT_MAX);
  DPS_LAUNCHED();
  if (n_px_cap == 0) return DPS_OK;
  DPS_REQUIRE(px_paper && px_mid, DPS_ERR_INVALID, "null PX pairs");
  k_paper_mid_pairs<<<grid_for(n_px_cap, kBlock), kBlock, 0, st>>>(px_paper, px_mid, n_px_cap,
                                                                   n_px_dev, vp);
  DPS_LAUNCHED();
  return DPS_OK;
}

int dps_spgemm_single(const int64_t* ap_ptr, const int32_t* ap_col, int64_t n_out_rows,
                      int64_t nnz_ap_cap, const int64_t* px_ptr, const int32_t* px_col,
                      int64_t n_papers, int64_t n_mids, int64_t* c_ptr, int32_t* c_col,
                      int32_t* c_val, int64_t* c_nnz, void* ws, size_t ws_bytes, void* stream) {
  return dps_spgemm_single_map(ap_ptr, ap_col, n_out_rows, nnz_ap_cap, nullptr, px_ptr, px_col,
                               n_papers, n_mids, c_ptr, c_col, c_val, c_nnz, ws, ws_bytes, stream);
}

int dps_spgemm_single_map(const int64_t* ap_ptr, const int32_t* ap_col, int64_t n_out_rows,
                          int64_t nnz_ap_cap, const int32_t* vp_in, const int64_t* px_ptr,
                          const int32_t* px_col, int64_t n_papers, int64_t n_mids,
                          int64_t* c_ptr, int32_t* c_col, int32_t* c_val, int64_t* c_nnz,
                          void* ws, size_t ws_bytes, void* stream) {
  DPS_REQUIRE(n_out_rows >= 0 && nnz_ap_cap >= 0, DPS_ERR_INVALID, "negative size");
  DPS_REQUIRE(c_ptr && c_nnz, DPS_ERR_INVALID, "null output");
  DPS_REQUIRE(!c_col == !c_val, DPS_ERR_INVALID, "c_col and c_val must both be set (numeric)");
  DPS_REQUIRE(reinterpret_cast<uintptr_t>(ws) % 256 == 0, DPS_ERR_WORKSPACE,
              "workspace not 256-byte aligned");
  DPS_REQUIRE(n_papers >= 0 && n_mids >= 0, DPS_ERR_INVALID, "negative n_papers / n_mids");
  DPS_REQUIRE(ws_bytes >= dps_spgemm_single_workspace_size(n_out_rows, nnz_ap_cap, n_papers),
              DPS_ERR_WORKSPACE, "spgemm_single workspace too small");
  auto st = static_cast<hipStream_t>(stream);
  Carve c(ws, ws_bytes);
  const int64_t n = n_out_rows > 0 ? n_out_rows : 1;
  int32_t* vp = c.take<int32_t>(n_papers > 0 ? n_papers : 1);
  int32_t* mids = c.take<int32_t>(nnz_ap_cap > 0 ? nnz_ap_cap : 1);
  int32_t* cnt = c.take<int32_t>(nnz_ap_cap > 0 ? nnz_ap_cap : 1);
  int64_t* uniq = c.take<int64_t>(n);
  const size_t scan_ws = scan_workspace_size(n_out_rows + 1);
  void* sws = c.take<char>(scan_ws);
  const size_t seg_ws = seg_unique_workspace_size(n_out_rows);
  void* gws = c.take<char>(seg_ws);
  DPS_REQUIRE(c.ok, DPS_ERR_WORKSPACE, "spgemm_single workspace carve failed");
  if (c_col == nullptr) {   // symbolic: map, segmented sort + unique, scan
    if (n_out_rows > 0) {
      if (vp_in) {
        vp = const_cast<int32_t*>(vp_in);
      } else if (n_papers > 0) {
        DPS_REQUIRE(px_ptr && px_col, DPS_ERR_INVALID, "px_ptr / px_col (or vp) required");
        k_paper_mid<<<grid_for(n_papers, kBlock), kBlock, 0, st>>>(px_ptr, px_col, n_papers, vp);
        DPS_LAUNCHED();
      }
      // the paper -> mid gather happens in the segmented sort's loads
      // (SegSrc): mids is written only with each row's distinct mids
      SegSrc src;
      src.col = ap_col;
      src.map = vp;
      DPS_HIP_RET(seg_unique(mids, cnt, ap_ptr, n_out_rows, uniq, gws, seg_ws, st,
                             n_mids < INT32_MAX ? static_cast<int>(n_mids) : 0, src));
      k_drop_none<<<grid_for(n_out_rows, kBlock), kBlock, 0, st>>>(mids, ap_ptr, n_out_rows, uniq);
      DPS_LAUNCHED();
    }
    DPS_HIP_RET(scan_exclusive<int64_t>(uniq, c_ptr, n_out_rows, sws, scan_ws, st));
    k_total<<<1, 1, 0, st>>>(c_ptr, n_out_rows, c_nnz);
    DPS_LAUNCHED();
    return DPS_OK;
  }
  if (n_out_rows > 0) {
    k_compact_mids<<<grid_for(n_out_rows, kBlock), kBlock, 0, st>>>(mids, cnt, ap_ptr, c_ptr,
                                                                    n_out_rows, c_col, c_val);
    DPS_LAUNCHED();
  }
  return DPS_OK;
}

int dps_spgemm_hash(const int64_t* ap_ptr, const int32_t* ap_col, const int32_t* rows,
                    int64_t n_out_rows, const int64_t* px_ptr, const int32_t* px_col,
                    int64_t max_row_expand, int64_t* c_ptr, int32_t* c_col, int32_t* c_val,
                    int64_t* c_nnz, int32_t* status_dev, void* ws, size_t ws_bytes, void* stream) {
  DPS_REQUIRE(n_out_rows >= 0 && max_row_expand >= 0, DPS_ERR_INVALID, "negative size");
  DPS_REQUIRE(c_ptr && c_nnz, DPS_ERR_INVALID, "null output");
  DPS_REQUIRE(!c_col == !c_val, DPS_ERR_INVALID, "c_col and c_val must both be set (numeric)");
  DPS_REQUIRE(reinterpret_cast<uintptr_t>(ws) % 256 == 0, DPS_ERR_WORKSPACE,
              "workspace not 256-byte aligned");
  DPS_REQUIRE(ws_bytes >= dps_spgemm_hash_workspace_size(n_out_rows, max_row_expand),
              DPS_ERR_WORKSPACE, "spgemm_hash workspace too small");
  DPS_REQUIRE(max_row_expand < INT32_MAX, DPS_ERR_OVERFLOW, "row expansion exceeds int32");
  auto st = static_cast<hipStream_t>(stream);
  Carve c(ws, ws_bytes);
  const int64_t n = n_out_rows > 0 ? n_out_rows : 1;
  uint32_t* u = c.take<uint32_t>(n);
  int32_t* long_list = c.take<int32_t>(n);
  unsigned* n_long = c.take<unsigned>(4);
  const size_t scan_ws = scan_workspace_size(n_out_rows + 1);
  void* sws = c.take<char>(scan_ws);
  const int64_t hm = max_row_expand > kHashCap ? max_row_expand : 1;
  int32_t* huge = c.take<int32_t>(static_cast<size_t>(kHugeBlocks) * hm);
  DPS_REQUIRE(c.ok, DPS_ERR_WORKSPACE, "spgemm_hash workspace carve failed");
  const int grid_rows = grid_for(n_out_rows, kBlock);
  if (c_col == nullptr) {   // symbolic: u, long rows, c_ptr, c_nnz
    if (status_dev) DPS_HIP_RET(hipMemsetAsync(status_dev, 0, sizeof(int32_t), st));
    DPS_HIP_RET(hipMemsetAsync(n_long, 0, sizeof(unsigned), st));
    if (n_out_rows > 0) {
      k_hash_rows<false><<<grid_rows, kBlock, 0, st>>>(ap_ptr, ap_col, rows, n_out_rows, px_ptr,
                                                      px_col, u, long_list, n_long, nullptr,
                                                      nullptr, nullptr);
      DPS_LAUNCHED();
      k_hash_long<false><<<512, kBlock, 0, st>>>(ap_ptr, ap_col, rows, px_ptr, px_col, u,
                                                 long_list, n_long, nullptr, nullptr, nullptr,
                                                 huge, hm, status_dev);
      DPS_LAUNCHED();
    }
    DPS_HIP_RET(scan_exclusive<uint32_t>(u, c_ptr, n_out_rows, sws, scan_ws, st));
    k_total<<<1, 1, 0, st>>>(c_ptr, n_out_rows, c_nnz);
    DPS_LAUNCHED();
    return DPS_OK;
  }
  // numeric (the workspace of the preceding symbolic call, unmodified)
  if (n_out_rows > 0) {
    k_hash_rows<true><<<grid_rows, kBlock, 0, st>>>(ap_ptr, ap_col, rows, n_out_rows, px_ptr,
                                                   px_col, u, long_list, n_long, c_ptr, c_col,
                                                   c_val);
    DPS_LAUNCHED();
    k_hash_long<true><<<512, kBlock, 0, st>>>(ap_ptr, ap_col, rows, px_ptr, px_col, u, long_list,
                                              n_long, c_ptr, c_col, c_val, huge, hm, status_dev);
    DPS_LAUNCHED();
  }
  return DPS_OK;
}

}  // extern "C"
