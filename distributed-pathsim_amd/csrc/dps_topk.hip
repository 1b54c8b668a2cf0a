// ★ Hot path: target-tiled C.C^T with the fused fp64 PathSim epilogue and a
// per-source top-k, plus the single-source row and
// pair kernels used by the reference-compatible class.
//
// Layout (see DESIGN.md "Data layout in HBM"):
//   C       : CSR over author rows, int64 row_ptr / int32 col / int32 val.
//   tiles   : C^T cut into target tiles of W = 2^shift authors; bucket (v,t)
//             holds packed uint32 entries (C[y,v] << 16) | (y - t*W), buckets
//             stored [v][t] so one row's venue v walks its buckets in order.
// Kernel (one wave64 per workgroup, persistent, rows dequeued in chunks):
//   for each source row x, for each target tile t:
//     scatter   acc[y_l] += C[x,v]*C[y,v] (LDS int32, no-return ds_add) and
//               mark y_l in an LDS bitmap,
//     compact   bitmap -> list of touched y_l (wave prefix sum),
//     epilogue  reject M < mmin (integer bound, no g load), else
//               score = double(2M)/double(gx+gy) -- one IEEE division, the
//               reference's :51-52 -- and insert into the register-resident
//               top-k (lane i holds rank i, KPL ranks per lane).
#include "dps_common.hpp"

#include <cstdlib>

namespace dps {
namespace {

constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kRowChunk = 4;  // rows per dequeue

// --------------------------------------------------------------------------
// Target relabeling: ascending global walk g (ties: original index).  Tiles of
// consecutive labels then hold targets of near-equal g, so a per-tile lower
// bound gmin_t on g[y] makes the score filter almost exact.
__global__ __launch_bounds__(kBlock) void k_invert_perm(const uint32_t* __restrict__ perm,
                                                        int64_t n, int32_t* __restrict__ rank) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * kBlock)
    rank[perm[i]] = static_cast<int32_t>(i);
}

// --------------------------------------------------------------------------
// Tile build: counting sort of C entries into (v, t) buckets, t = label >> shift.
__device__ __forceinline__ int64_t label_of(const int32_t* rank, int64_t y) {
  return rank ? static_cast<int64_t>(rank[y]) : y;
}

__global__ __launch_bounds__(kBlock) void k_tile_count(const int64_t* __restrict__ c_ptr,
                                                       const int32_t* __restrict__ c_col,
                                                       const int32_t* __restrict__ c_val,
                                                       const int32_t* __restrict__ rank,
                                                       const int64_t* __restrict__ g,
                                                       int64_t n_rows, int shift, int64_t T,
                                                       uint32_t* __restrict__ cnt,
                                                       uint32_t* __restrict__ maxc,
                                                       unsigned long long* __restrict__ gmin,
                                                       int32_t* __restrict__ status) {
  const int lane = lane_id();
  const int64_t wave0 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWavesPerBlock;
  for (int64_t y = wave0; y < n_rows; y += nwaves) {
    const int64_t t = label_of(rank, y) >> shift;
    if (lane == 0 && gmin) atomicMin(&gmin[t], static_cast<unsigned long long>(g[y]));
    for (int64_t j = c_ptr[y] + lane; j < c_ptr[y + 1]; j += kWave) {
      const int32_t c = c_val[j];
      if (c > 0xFFFF && status) *status = DPS_ERR_OVERFLOW;
      const int64_t b = static_cast<int64_t>(c_col[j]) * T + t;
      atomicAdd(&cnt[b], 1u);
      if (maxc) atomicMax(&maxc[b], static_cast<uint32_t>(c));
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_tile_off32(const int64_t* __restrict__ p64,
                                                       int64_t n, uint32_t* __restrict__ p32) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i <= n;
       i += static_cast<int64_t>(gridDim.x) * kBlock)
    p32[i] = static_cast<uint32_t>(p64[i]);
}

__global__ __launch_bounds__(kBlock) void k_tile_scatter(const int64_t* __restrict__ c_ptr,
                                                         const int32_t* __restrict__ c_col,
                                                         const int32_t* __restrict__ c_val,
                                                         const int32_t* __restrict__ rank,
                                                         int64_t n_rows, int shift, int64_t T,
                                                         const int64_t* __restrict__ off,
                                                         uint32_t* __restrict__ cursor,
                                                         uint32_t* __restrict__ ent) {
  const int lane = lane_id();
  const int64_t wave0 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWavesPerBlock;
  const uint32_t ymask = (1u << shift) - 1u;
  for (int64_t y = wave0; y < n_rows; y += nwaves) {
    const int64_t lab = label_of(rank, y);
    const int64_t t = lab >> shift;
    for (int64_t j = c_ptr[y] + lane; j < c_ptr[y + 1]; j += kWave) {
      const int64_t b = static_cast<int64_t>(c_col[j]) * T + t;
      const uint32_t pos = atomicAdd(&cursor[b], 1u);
      ent[off[b] + pos] =
          (static_cast<uint32_t>(c_val[j]) << 16) | (static_cast<uint32_t>(lab) & ymask);
    }
  }
}

// --------------------------------------------------------------------------
// Top-k helpers.  Order: score desc, then ORIGINAL target index asc.
__device__ __forceinline__ bool better(double s1, int y1, double s2, int y2) {
  return s1 > s2 || (s1 == s2 && y1 < y2);
}

// Smallest m >= 0 with fl(2m / den) >= kth (den > 0).  For every target y of a
// tile, gx + g[y] >= den := gx + gmin_t, so fl(2M/(gx+g[y])) <= fl(2M/den)
// (rounding is monotone) and m -> 2m/den is increasing: a candidate with
// M < mneed scores strictly below the current k-th and is rejected with one
// integer compare -- no g load, no division.
__device__ int compute_mneed(double kth, int64_t den) {
  if (kth <= 0.0 || den <= 0) return 0;
  int64_t m = static_cast<int64_t>(kth * static_cast<double>(den) * 0.5) - 2;
  if (m < 0) m = 0;
  const double dd = static_cast<double>(den);
  while (static_cast<double>(2 * m) / dd < kth) ++m;
  while (m > 0 && static_cast<double>(2 * (m - 1)) / dd >= kth) --m;
  return m > INT32_MAX ? INT32_MAX : static_cast<int>(m);
}

template <int KPL>
struct TopK {
  double s[KPL];
  int y[KPL];
  int m[KPL];
  int k;
  int filled;
  double kth_s;
  int kth_y;

  __device__ void init(int k_) {
#pragma unroll
    for (int r = 0; r < KPL; ++r) { s[r] = -1.0; y[r] = INT_MAX; m[r] = 0; }
    k = k_;
    filled = 0;
    kth_s = -1.0;
    kth_y = INT_MAX;
  }
  __device__ bool full() const { return filled == k; }
  // Insert a candidate already known to beat the k-th entry (wave-uniform args).
  __device__ void insert(double cs, int cy, int cm) {
    const int lane = lane_id();
    int pos = 0;
#pragma unroll
    for (int r = 0; r < KPL; ++r) {
      const bool b = (r * kWave + lane < k) && better(s[r], y[r], cs, cy);
      pos += __popcll(ballot(b));
    }
    double us[KPL];
    int uy[KPL], um[KPL];
#pragma unroll
    for (int r = 0; r < KPL; ++r) {
      us[r] = __shfl_up(s[r], 1, kWave);
      uy[r] = __shfl_up(y[r], 1, kWave);
      um[r] = __shfl_up(m[r], 1, kWave);
      if (r > 0 && lane == 0) {
        us[r] = readlane(s[r - 1], kWave - 1);
        uy[r] = readlane(y[r - 1], kWave - 1);
        um[r] = readlane(m[r - 1], kWave - 1);
      }
    }
#pragma unroll
    for (int r = 0; r < KPL; ++r) {
      const int slot = r * kWave + lane;
      if (slot > pos) { s[r] = us[r]; y[r] = uy[r]; m[r] = um[r]; }
      else if (slot == pos) { s[r] = cs; y[r] = cy; m[r] = cm; }
    }
    filled = filled < k ? filled + 1 : k;
    const int rk = (k - 1) / kWave, lk = (k - 1) % kWave;
#pragma unroll
    for (int r = 0; r < KPL; ++r)
      if (r == rk) { kth_s = readlane(s[r], lk); kth_y = readlane(y[r], lk); }
  }
};

struct HotParams {
  const int64_t* c_ptr;
  const int32_t* c_col;
  const int32_t* c_val;
  const int64_t* g;          // original order (sources)
  const int64_t* g_t;        // target label order
  const int32_t* t_perm;     // label -> original (nullable = identity)
  const int32_t* t_rank;     // original -> label (nullable = identity)
  const uint32_t* tile_off;
  const uint32_t* tile_ent;
  const uint32_t* tile_maxc; // never null in the kernel (tile_off stands in)
  bool use_maxc;             // false: no tile skipping
  const int64_t* tile_gmin;
  int64_t n_targets;
  int64_t T;
  int shift;
  int64_t row_begin;
  int64_t n_rows;
  int k;
  int32_t* out_idx;
  int64_t* out_cnt;
  double* out_score;
  unsigned long long* counter;
  int ablate;  // profiling aid (DPATHSIM_ABLATE): 1 no LDS atomics, 2 no epilogue, 4 no scatter
};

__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave-uniform read-only loads through the constant address space: hipcc
// emits s_load (lgkmcnt) instead of a vector load, so they never force a
// vmcnt(0) that would drain the next tile's chunk loads.
template <class T>
__device__ __forceinline__ T ld_uniform(const T* p, int64_t i) {
  typedef const __attribute__((address_space(4))) T* cptr;
  return ((cptr)(reinterpret_cast<uintptr_t>(p)))[i];
}

constexpr int kCandCap = 512;   // crossing-candidate list capacity per wave (uint16)
constexpr int kChunksPL = 4;    // 16-byte chunks per lane kept in flight per tile unit
constexpr int kPre = 4;         // tile-bound prefetch distance

// Per-wave scatter state for one (row, tile).  acc[y] accumulates M; the
// returned old value drives two wave-private lists (no LDS atomics besides the
// add): `tl` = targets touched for the first time (cleared after the tile),
// `cl` = targets whose running M crossed `me` (the tile's candidates).
struct Scatter {
  int32_t* acc;
  uint16_t* tl;
  uint16_t* cl;
  int me;         // crossing threshold (>= 1)
  int n_t;        // touched count (wave-uniform)
  int n_c;        // candidate count (wave-uniform)
  bool track_c;   // false: every touched target is a candidate (tl doubles as cl)
  int ablate;

  __device__ __forceinline__ void add(bool valid, uint32_t e, int c) {
    const int yl = static_cast<int>(e & 0xFFFFu);
    const int inc = c * static_cast<int>(e >> 16);
    int old = 1;
    if (valid) {
      if (ablate & 1) old = 1 + (yl & 0);
      else old = atomicAdd(&acc[yl], inc);
    }
    const bool fresh = valid && old == 0;
    const uint64_t mt = ballot(fresh);
    if (fresh) tl[n_t + mbcnt(mt)] = static_cast<uint16_t>(yl);
    n_t += __popcll(mt);
    if (track_c) {
      const bool cross = valid && old < me && old + inc >= me;
      const uint64_t mc = ballot(cross);
      if (cross) {
        const int pos = n_c + mbcnt(mc);
        if (pos < kCandCap) cl[pos] = static_cast<uint16_t>(yl);
      }
      n_c += __popcll(mc);
    }
  }
};

// One tile "unit" of a row: its buckets flattened into 16-byte chunks.  Lane j
// describes venue j's bucket [lo, hi) and multiplier c; chunk q of the unit is
// located by a wave binary search over the exclusive chunk prefix `pre`.
struct Unit {
  uint32_t lo, hi;   // lane j: bucket bounds (entries)
  int c;             // lane j: C[x, v_j]
  int pre;           // lane j: exclusive prefix of chunk counts
  int nq;            // total chunks (wave-uniform)
  uint4 e[kChunksPL];
  int jq[kChunksPL]; // venue of each held chunk (-1: none)
};

__device__ __forceinline__ int chunk_venue(int pre, int q) {
  int j = 0;
#pragma unroll
  for (int step = kWave / 2; step > 0; step >>= 1) {
    const int cand = j + step;
    const int pv = __shfl(pre, cand & (kWave - 1), kWave);
    if (cand < kWave && pv <= q) j = cand;
  }
  return j;
}

__device__ __forceinline__ uint32_t chunk_base(const Unit& U, int j, int q) {
  const uint32_t a0 = __shfl(static_cast<int>(U.lo & ~3u), j, kWave);
  const int pj = __shfl(U.pre, j, kWave);
  return a0 + 4u * static_cast<uint32_t>(q - pj);
}

// Describe the unit and issue the loads of its first kChunksPL*64 chunks.
// Branch-free on purpose: every lane issues every load (out-of-range chunks
// read entry 0), so hipcc can count the loads and wait with vmcnt(N) instead
// of draining the next unit's loads (vmcnt(0)) when this one is consumed.
__device__ __forceinline__ void unit_issue(Unit& U, const uint32_t* __restrict__ ent, uint32_t lo,
                                           uint32_t hi, int c, int lane) {
  U.lo = lo;
  U.hi = hi;
  U.c = c;
  const int nch = hi > lo ? static_cast<int>((hi - (lo & ~3u) + 3u) >> 2) : 0;
  const int inc = wave_inclusive_sum(nch);
  U.pre = inc - nch;
  U.nq = readlane(inc, kWave - 1);
#pragma unroll
  for (int u = 0; u < kChunksPL; ++u) {
    const int q = u * kWave + lane;
    const int j = chunk_venue(U.pre, q);
    const bool live = q < U.nq;
    // the shuffles inside chunk_base must run in every lane (a bpermute from
    // an inactive source lane returns garbage): compute, then select
    const uint32_t b = chunk_base(U, j, q);
    const uint32_t base = live ? b : 0u;
    U.e[u] = *reinterpret_cast<const uint4*>(ent + base);
    U.jq[u] = live ? j : -1;
  }
}

__device__ __forceinline__ void chunk_add(Scatter& S, const Unit& U, uint4 e, int j, int q) {
  // bounds / multiplier of the chunk's venue (j wave-varying -> bpermute)
  const int jj = j < 0 ? 0 : j;
  const uint32_t lo = static_cast<uint32_t>(__shfl(static_cast<int>(U.lo), jj, kWave));
  const uint32_t hi = static_cast<uint32_t>(__shfl(static_cast<int>(U.hi), jj, kWave));
  const int c = __shfl(U.c, jj, kWave);
  const int pj = __shfl(U.pre, jj, kWave);
  const uint32_t base = (lo & ~3u) + 4u * static_cast<uint32_t>(q - pj);
  const bool ok = j >= 0;
  S.add(ok && base >= lo && base < hi, e.x, c);
  S.add(ok && base + 1 >= lo && base + 1 < hi, e.y, c);
  S.add(ok && base + 2 >= lo && base + 2 < hi, e.z, c);
  S.add(ok && base + 3 >= lo && base + 3 < hi, e.w, c);
}

// Scatter everything of the unit: held chunks first, then any remainder.
__device__ __forceinline__ uint32_t unit_process(Scatter& S, const Unit& U,
                                                 const uint32_t* __restrict__ ent, int lane) {
  if (U.nq == 0) return 0;
#pragma unroll
  for (int u = 0; u < kChunksPL; ++u)
    if (u * kWave < U.nq) chunk_add(S, U, U.e[u], U.jq[u], u * kWave + lane);
  for (int q0 = kChunksPL * kWave; q0 < U.nq; q0 += kWave) {   // rare: large units
    const int q = q0 + lane;
    const int j = chunk_venue(U.pre, q);
    const uint32_t base = chunk_base(U, j, q);
    uint4 e = make_uint4(0, 0, 0, 0);
    if (q < U.nq) e = *reinterpret_cast<const uint4*>(ent + base);
    chunk_add(S, U, e, q < U.nq ? j : -1, q);
  }
  return static_cast<uint32_t>(U.nq);
}

// Candidates of one tile: exact score for the survivors of the integer filter,
// then clear the touched accumulators.
template <int KPL>
__device__ __forceinline__ void tile_epilogue(const HotParams& p, Scatter& S, TopK<KPL>& top,
                                              int64_t t, int mneed, int64_t x_lab, int64_t gx,
                                              int lane) {
  wave_lds_fence();
  const bool from_tl = !S.track_c || S.n_c > kCandCap;   // overflow: rescan touched
  const uint16_t* src = from_tl ? S.tl : S.cl;
  const int n_src = from_tl ? S.n_t : S.n_c;
  const int64_t y0 = t << p.shift;
  for (int i0 = 0; i0 < n_src; i0 += kWave) {
    const int i = i0 + lane;
    int yl = 0, M = 0;
    if (i < n_src) {
      yl = src[i];
      M = S.acc[yl];
    }
    const int64_t ylab = y0 + yl;
    bool cand = (i < n_src) && (M >= mneed) && (ylab != x_lab);
    double sc = 0.0;
    int yo = 0;
    if (cand) {
      yo = p.t_perm ? p.t_perm[ylab] : static_cast<int>(ylab);
      const int64_t den = gx + p.g_t[ylab];
      sc = den ? static_cast<double>(2 * static_cast<int64_t>(M)) / static_cast<double>(den) : 0.0;
      cand = better(sc, yo, top.kth_s, top.kth_y);
    }
    uint64_t mask = ballot(cand);
    while (mask) {
      const int srcl = __ffsll(static_cast<long long>(mask)) - 1;
      mask &= mask - 1;
      const double cs = readlane(sc, srcl);
      const int cy = readlane(yo, srcl);
      if (!better(cs, cy, top.kth_s, top.kth_y)) continue;
      top.insert(cs, cy, readlane(M, srcl));
    }
  }
  wave_lds_fence();
  for (int i = lane; i < S.n_t; i += kWave) S.acc[S.tl[i]] = 0;
  wave_lds_fence();
}

// Per-wave LDS image: acc int32[W] | touched uint16[W] | candidates uint16[kCandCap].
template <int KPL>
__global__ __launch_bounds__(kWave) void k_cct_topk(HotParams p) {
  extern __shared__ __attribute__((aligned(16))) int32_t lds[];
  const int lane = threadIdx.x;
  const int W = 1 << p.shift;
  int32_t* acc = lds;
  uint16_t* tl = reinterpret_cast<uint16_t*>(lds + W);
  uint16_t* cl = tl + W;

  for (int i = lane; i < W; i += kWave) acc[i] = 0;
  wave_lds_fence();

  for (;;) {
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(p.counter, static_cast<unsigned long long>(kRowChunk));
    base = __shfl(base, 0, kWave);
    if (static_cast<int64_t>(base) >= p.n_rows) break;
    const int64_t r_end = min(static_cast<int64_t>(base) + kRowChunk, p.n_rows);
    for (int64_t r = static_cast<int64_t>(base); r < r_end; ++r) {
      const int64_t x = p.row_begin + r;
      const int64_t x_lab = p.t_rank ? static_cast<int64_t>(ld_uniform(p.t_rank, x)) : x;
      const int64_t pb = ld_uniform(p.c_ptr, x);
      const int d = static_cast<int>(ld_uniform(p.c_ptr, x + 1) - pb);
      const int64_t gx = ld_uniform(p.g, x);
      TopK<KPL> top;
      top.init(p.k);
      Scatter S;
      S.acc = acc; S.tl = tl; S.cl = cl; S.ablate = p.ablate;

      if (d > 0 && d <= kWave) {
        // ---- fast path: lane j keeps venue j; bucket ends / maxima are
        // prefetched kPre tiles ahead and each tile's chunks are loaded one
        // tile ahead (unit `nx` in flight while unit `cu` is scattered).
        int v_reg = 0, c_reg = 0;
        uint32_t lo_reg = 0, hi_q[kPre], mx_q[kPre];
#pragma unroll
        for (int q = 0; q < kPre; ++q) { hi_q[q] = 0; mx_q[q] = 0; }
        if (lane < d) {
          v_reg = p.c_col[pb + lane];
          c_reg = p.c_val[pb + lane];
        }
        {
          const int64_t vb = static_cast<int64_t>(v_reg) * p.T;   // lanes >= d: venue 0, c 0
          lo_reg = p.tile_off[vb];
#pragma unroll
          for (int q = 0; q < kPre; ++q) {
            const int64_t tq = min(static_cast<int64_t>(q), p.T - 1);
            hi_q[q] = p.tile_off[vb + tq + 1];
            mx_q[q] = p.tile_maxc[vb + tq];
          }
          if (lane >= d) {      // lanes without a venue hold empty buckets
            lo_reg = 0;
#pragma unroll
            for (int q = 0; q < kPre; ++q) hi_q[q] = 0;
          }
        }
        Unit cu, nx;
        bool cu_live = false;
        {
          const bool skip0 = (p.ablate & 4) != 0;
          unit_issue(cu, p.tile_ent, lo_reg, skip0 ? lo_reg : hi_q[0], c_reg, lane);
          cu_live = true;
        }
        for (int64_t t = 0; t < p.T; ++t) {
          int mneed = 0;
          if (top.full()) mneed = compute_mneed(top.kth_s, gx + ld_uniform(p.tile_gmin, t));
          const uint32_t hi_t = hi_q[0], mx_t = mx_q[0];
          // the next tile's bucket bounds are hi_t .. hi_q[1]: issue its loads now
          const uint32_t hi_n = hi_q[1];
#pragma unroll
          for (int q = 0; q + 1 < kPre; ++q) { hi_q[q] = hi_q[q + 1]; mx_q[q] = mx_q[q + 1]; }
          {  // unconditional (clamped) prefetch of tile t + kPre
            const int64_t tp = min(t + kPre, p.T - 1);
            const int64_t vb = static_cast<int64_t>(v_reg) * p.T + tp;
            const uint32_t hv = p.tile_off[vb + 1];
            hi_q[kPre - 1] = lane < d ? hv : 0u;
            mx_q[kPre - 1] = p.tile_maxc[vb];
          }
          bool skip = (p.ablate & 4) != 0;
          if (mneed > 0 && p.use_maxc)
            skip = skip || wave_sum(static_cast<int64_t>(c_reg) * mx_t) < mneed;
#ifndef DPS_NO_PIPELINE
          unit_issue(nx, p.tile_ent, hi_t, (p.ablate & 4) || t + 1 >= p.T ? hi_t : hi_n, c_reg,
                     lane);
#endif
          S.me = mneed > 1 ? mneed : 1;
          S.track_c = top.full();
          S.n_t = 0;
          S.n_c = 0;
          uint32_t scattered = 0;
          if (!skip && cu_live) scattered = unit_process(S, cu, p.tile_ent, lane);
#ifdef DPS_NO_PIPELINE
          unit_issue(nx, p.tile_ent, hi_t, (p.ablate & 4) || t + 1 >= p.T ? hi_t : hi_n, c_reg,
                     lane);
#endif
          cu = nx;
          cu_live = t + 1 < p.T;
          lo_reg = hi_t;
          if (scattered == 0) continue;
          if (p.ablate & 2) {
            wave_lds_fence();
            for (int i = lane; i < S.n_t; i += kWave) acc[tl[i]] = 0;
            wave_lds_fence();
            continue;
          }
          tile_epilogue<KPL>(p, S, top, t, mneed, x_lab, gx, lane);
        }
      } else if (d > kWave) {
        // ---- general path (> 64 venues): 64-venue chunks, no pipelining ----
        for (int64_t t = 0; t < p.T; ++t) {
          const int64_t gmin_t = ld_uniform(p.tile_gmin, t);
          int mneed = 0;
          if (top.full()) mneed = compute_mneed(top.kth_s, gx + gmin_t);
          bool skip = (p.ablate & 4) != 0;
          if (mneed > 0 && p.use_maxc) {
            int64_t ub = 0;
            for (int c0 = 0; c0 < d; c0 += kWave) {
              const int j = c0 + lane;
              if (j < d)
                ub += static_cast<int64_t>(p.c_val[pb + j]) *
                      p.tile_maxc[static_cast<int64_t>(p.c_col[pb + j]) * p.T + t];
            }
            skip = skip || wave_sum(ub) < mneed;
          }
          S.me = mneed > 1 ? mneed : 1;
          S.track_c = top.full();
          S.n_t = 0;
          S.n_c = 0;
          uint32_t scattered = 0;
          for (int c0 = 0; !skip && c0 < d; c0 += kWave) {
            const int j = c0 + lane;
            int cx = 0;
            uint32_t lo = 0, hi = 0;
            if (j < d) {
              const int64_t vb = static_cast<int64_t>(p.c_col[pb + j]) * p.T + t;
              cx = p.c_val[pb + j];
              lo = p.tile_off[vb];
              hi = p.tile_off[vb + 1];
            }
            Unit U;
            unit_issue(U, p.tile_ent, lo, hi, cx, lane);
            scattered += unit_process(S, U, p.tile_ent, lane);
          }
          if (scattered == 0) continue;
          if (p.ablate & 2) {
            wave_lds_fence();
            for (int i = lane; i < S.n_t; i += kWave) acc[tl[i]] = 0;
            wave_lds_fence();
            continue;
          }
          tile_epilogue<KPL>(p, S, top, t, mneed, x_lab, gx, lane);
        }
      }
      // ---- write: ranked entries, zero-score fill, empty slots --------------
      int32_t* oi = p.out_idx + r * p.k;
      int64_t* oc = p.out_cnt + r * p.k;
      double* os = p.out_score + r * p.k;
#pragma unroll
      for (int q = 0; q < KPL; ++q) {
        const int slot = q * kWave + lane;
        if (slot < top.filled) { oi[slot] = top.y[q]; oc[slot] = top.m[q]; os[slot] = top.s[q]; }
      }
      const int64_t avail = p.n_targets - 1;
      const int want = static_cast<int>(avail < p.k ? avail : p.k);
      int slot = top.filled;
      for (int64_t yb = 0; slot < want && yb < p.n_targets; yb += kWave) {
        const int64_t yc = yb + lane;
        bool ok = yc < p.n_targets && yc != x;
        for (int q = 0; q < KPL; ++q) {
          for (int l = 0; l < kWave; ++l) {
            if (q * kWave + l >= top.filled) break;
            ok = ok && (readlane(top.y[q], l) != static_cast<int>(yc));
          }
        }
        const uint64_t mk = ballot(ok);
        const int rank = mbcnt(mk);
        if (ok && slot + rank < want) {
          oi[slot + rank] = static_cast<int32_t>(yc);
          oc[slot + rank] = 0;
          os[slot + rank] = 0.0;
        }
        slot += __popcll(mk);
      }
      for (int s2 = want + lane; s2 < p.k; s2 += kWave) {
        oi[s2] = -1;
        oc[s2] = 0;
        os[s2] = 0.0;
      }
    }
  }
}

// --------------------------------------------------------------------------
// Single-source dense row: one block per target tile; out_m in ORIGINAL order.
__global__ __launch_bounds__(kBlock) void k_walk_row(const int32_t* __restrict__ src_col,
                                                     const int32_t* __restrict__ src_val,
                                                     int64_t src_len, int64_t n_targets, int shift,
                                                     int64_t T, const uint32_t* __restrict__ off,
                                                     const uint32_t* __restrict__ ent,
                                                     const int32_t* __restrict__ t_perm,
                                                     int64_t* __restrict__ out_m) {
  extern __shared__ __attribute__((aligned(16))) int32_t acc[];
  const int W = 1 << shift;
  const int64_t t = blockIdx.x;
  for (int i = threadIdx.x; i < W; i += kBlock) acc[i] = 0;
  __syncthreads();
  for (int64_t j = 0; j < src_len; ++j) {
    const int64_t b = static_cast<int64_t>(src_col[j]) * T + t;
    const int cx = src_val[j];
    for (uint32_t i = off[b] + threadIdx.x; i < off[b + 1]; i += kBlock) {
      const uint32_t e = ent[i];
      atomicAdd(&acc[e & 0xFFFFu], cx * static_cast<int>(e >> 16));
    }
  }
  __syncthreads();
  const int64_t y0 = t << shift;
  for (int i = threadIdx.x; i < W && y0 + i < n_targets; i += kBlock) {
    const int64_t lab = y0 + i;
    out_m[t_perm ? t_perm[lab] : lab] = acc[i];
  }
}

// score[y] = (double)(2*m[y]) / (double)(gx + g[y]) -- the reference's :51-52
// for one source row; *zero_div = number of targets with gx + g[y] == 0
// (the reference raises ZeroDivisionError there; score is left 0.0).
__global__ __launch_bounds__(kBlock) void k_row_scores(const int64_t* __restrict__ m,
                                                       const int64_t* __restrict__ g, int64_t gx,
                                                       int64_t n, double* __restrict__ score,
                                                       unsigned long long* zero_div) {
  for (int64_t y = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; y < n;
       y += static_cast<int64_t>(gridDim.x) * kBlock) {
    const int64_t den = gx + g[y];
    if (den == 0) {
      score[y] = 0.0;
      if (zero_div) atomicAdd(zero_div, 1ull);
    } else {
      score[y] = static_cast<double>(2 * m[y]) / static_cast<double>(den);
    }
  }
}

__global__ __launch_bounds__(kWave) void k_pair_count(const int32_t* __restrict__ a_col,
                                                      const int32_t* __restrict__ a_val,
                                                      int64_t a_len,
                                                      const int32_t* __restrict__ b_col,
                                                      const int32_t* __restrict__ b_val,
                                                      int64_t b_len, int64_t* out) {
  int64_t sum = 0;
  for (int64_t i = threadIdx.x; i < a_len; i += kWave) {
    const int32_t v = a_col[i];
    int64_t lo = 0, hi = b_len;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (b_col[mid] < v) lo = mid + 1; else hi = mid;
    }
    if (lo < b_len && b_col[lo] == v) sum += static_cast<int64_t>(a_val[i]) * b_val[lo];
  }
  sum = wave_sum(sum);
  if (threadIdx.x == 0) *out = sum;
}

int log2_exact(int32_t w) {
  int s = 0;
  while (s < 31 && (1 << s) < w) ++s;
  return (1 << s) == w ? s : -1;
}

}  // namespace
}  // namespace dps

using namespace dps;

static size_t hot_lds_bytes(int shift) {
  const size_t W = size_t(1) << shift;
  return W * sizeof(int32_t) + W * sizeof(uint16_t) + kCandCap * sizeof(uint16_t);
}

template <int KPL>
static int launch_hot(const HotParams& p, size_t lds, int64_t grid, hipStream_t st) {
  DPS_HIP_RET(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_cct_topk<KPL>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  static_cast<int>(lds)));
  k_cct_topk<KPL><<<static_cast<unsigned>(grid), kWave, lds, st>>>(p);
  DPS_LAUNCHED();
  return DPS_OK;
}


extern "C" {

size_t dps_target_order_workspace_size(int64_t n_targets) {
  return radix_sort_workspace_size(n_targets);
}

int dps_target_order(const int64_t* g, int64_t n_targets, int32_t key_bits, int32_t* t_perm,
                     int32_t* t_rank, int64_t* g_t, void* ws, size_t ws_bytes, void* stream) {
  DPS_REQUIRE(n_targets >= 0 && n_targets < INT32_MAX, DPS_ERR_INVALID, "bad n_targets");
  DPS_REQUIRE(key_bits >= 1 && key_bits <= 64, DPS_ERR_INVALID, "key_bits must be in [1,64]");
  DPS_REQUIRE(ws_bytes >= dps_target_order_workspace_size(n_targets), DPS_ERR_WORKSPACE,
              "target_order workspace too small");
  auto st = static_cast<hipStream_t>(stream);
  if (n_targets == 0) return DPS_OK;
  DPS_HIP_RET(radix_sort_pairs(reinterpret_cast<const uint64_t*>(g), nullptr,
                               reinterpret_cast<uint64_t*>(g_t),
                               reinterpret_cast<uint32_t*>(t_perm), n_targets, key_bits, ws,
                               ws_bytes, st));
  k_invert_perm<<<grid_for(n_targets, kBlock), kBlock, 0, st>>>(
      reinterpret_cast<const uint32_t*>(t_perm), n_targets, t_rank);
  DPS_LAUNCHED();
  return DPS_OK;
}

size_t dps_ct_tiles_workspace_size(int64_t n_mids, int64_t n_targets, int32_t tile_w) {
  if (tile_w <= 0) return 0;
  const int64_t T = (n_targets + tile_w - 1) / tile_w;
  const int64_t nb = n_mids * (T > 0 ? T : 1);
  size_t s = 0;
  s += align_up(static_cast<size_t>(nb + 1) * sizeof(uint32_t));  // cnt
  s += align_up(static_cast<size_t>(nb + 1) * sizeof(uint32_t));  // cursor
  s += align_up(static_cast<size_t>(nb + 1) * sizeof(int64_t));   // off64
  s += align_up(scan_workspace_size(nb + 1));
  return s + 1024;
}

int dps_ct_tiles_build(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                       const int64_t* g, const int32_t* t_rank, int64_t n_targets, int64_t n_mids,
                       int32_t tile_w, uint32_t* tile_off, uint32_t* tile_ent, uint32_t* tile_maxc,
                       int64_t* tile_gmin, int32_t* status_dev, void* ws, size_t ws_bytes,
                       void* stream) {
  const int shift = log2_exact(tile_w);
  DPS_REQUIRE(shift >= 8 && shift <= 14, DPS_ERR_UNSUPPORTED,
              "tile_w must be a power of two in [256, 16384], got %d", tile_w);
  DPS_REQUIRE(n_targets >= 0 && n_mids >= 0, DPS_ERR_INVALID, "negative size");
  DPS_REQUIRE(n_targets < INT32_MAX, DPS_ERR_OVERFLOW, "n_targets exceeds int32");
  DPS_REQUIRE(!tile_gmin || g, DPS_ERR_INVALID, "tile_gmin needs g");
  DPS_REQUIRE(reinterpret_cast<uintptr_t>(ws) % 256 == 0, DPS_ERR_WORKSPACE,
              "workspace not 256-byte aligned");
  DPS_REQUIRE(ws_bytes >= dps_ct_tiles_workspace_size(n_mids, n_targets, tile_w),
              DPS_ERR_WORKSPACE, "tiles workspace too small");
  auto st = static_cast<hipStream_t>(stream);
  const int64_t T = (n_targets + tile_w - 1) / tile_w;
  const int64_t nb = n_mids * T;
  Carve c(ws, ws_bytes);
  uint32_t* cnt = c.take<uint32_t>(nb + 1);
  uint32_t* cursor = c.take<uint32_t>(nb + 1);
  int64_t* off64 = c.take<int64_t>(nb + 1);
  const size_t scan_ws = scan_workspace_size(nb + 1);
  void* sws = c.take<char>(scan_ws);
  DPS_REQUIRE(c.ok, DPS_ERR_WORKSPACE, "tiles workspace carve failed");
  if (status_dev) DPS_HIP_RET(hipMemsetAsync(status_dev, 0, sizeof(int32_t), st));
  DPS_HIP_RET(hipMemsetAsync(cnt, 0, (nb + 1) * sizeof(uint32_t), st));
  DPS_HIP_RET(hipMemsetAsync(cursor, 0, (nb + 1) * sizeof(uint32_t), st));
  if (tile_maxc) DPS_HIP_RET(hipMemsetAsync(tile_maxc, 0, (nb + 1) * sizeof(uint32_t), st));
  if (tile_gmin && T > 0) DPS_HIP_RET(hipMemsetAsync(tile_gmin, 0x7F, T * sizeof(int64_t), st));
  if (n_targets > 0 && nb > 0) {
    k_tile_count<<<grid_for(n_targets * kWave, kBlock), kBlock, 0, st>>>(
        c_ptr, c_col, c_val, t_rank, g, n_targets, shift, T, cnt, tile_maxc,
        reinterpret_cast<unsigned long long*>(tile_gmin), status_dev);
    DPS_LAUNCHED();
  }
  DPS_HIP_RET(scan_exclusive<uint32_t>(cnt, off64, nb, sws, scan_ws, st));
  k_tile_off32<<<grid_for(nb + 1, kBlock), kBlock, 0, st>>>(off64, nb, tile_off);
  DPS_LAUNCHED();
  if (n_targets > 0 && nb > 0) {
    k_tile_scatter<<<grid_for(n_targets * kWave, kBlock), kBlock, 0, st>>>(
        c_ptr, c_col, c_val, t_rank, n_targets, shift, T, off64, cursor, tile_ent);
    DPS_LAUNCHED();
  }
  return DPS_OK;
}

size_t dps_cct_topk_workspace_size(void) { return 256; }

int dps_cct_topk(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                 const int64_t* g, const int64_t* g_t, const int32_t* t_perm,
                 const int32_t* t_rank, int64_t n_targets, int64_t n_mids, int32_t tile_w,
                 const uint32_t* tile_off, const uint32_t* tile_ent, const uint32_t* tile_maxc,
                 const int64_t* tile_gmin, int64_t row_begin, int64_t row_end, int32_t k,
                 int32_t* out_idx, int64_t* out_cnt, double* out_score, void* ws,
                 size_t ws_bytes, void* stream) {
  (void)n_mids;
  const int shift = log2_exact(tile_w);
  DPS_REQUIRE(shift >= 8 && shift <= 14, DPS_ERR_UNSUPPORTED,
              "tile_w must be a power of two in [256, 16384], got %d", tile_w);
  DPS_REQUIRE(k >= 1 && k <= 256, DPS_ERR_UNSUPPORTED, "k must be in [1, 256], got %d", k);
  DPS_REQUIRE(0 <= row_begin && row_begin <= row_end && row_end <= n_targets, DPS_ERR_INVALID,
              "row range [%lld, %lld) outside [0, %lld)", static_cast<long long>(row_begin),
              static_cast<long long>(row_end), static_cast<long long>(n_targets));
  DPS_REQUIRE(n_targets < INT32_MAX, DPS_ERR_OVERFLOW, "n_targets exceeds int32");
  DPS_REQUIRE(!t_perm == !t_rank, DPS_ERR_INVALID, "t_perm and t_rank go together");
  DPS_REQUIRE(tile_gmin && g, DPS_ERR_INVALID, "g and tile_gmin are required");
  DPS_REQUIRE(ws && ws_bytes >= dps_cct_topk_workspace_size(), DPS_ERR_WORKSPACE,
              "cct_topk workspace too small");
  auto st = static_cast<hipStream_t>(stream);
  const int64_t n_rows = row_end - row_begin;
  if (n_rows == 0) return DPS_OK;
  HotParams p;
  p.c_ptr = c_ptr; p.c_col = c_col; p.c_val = c_val;
  p.g = g; p.g_t = g_t ? g_t : g; p.t_perm = t_perm; p.t_rank = t_rank;
  p.tile_off = tile_off; p.tile_ent = tile_ent; p.tile_gmin = tile_gmin;
  p.tile_maxc = tile_maxc ? tile_maxc : tile_off;
  p.use_maxc = tile_maxc != nullptr;
  p.n_targets = n_targets;
  p.T = (n_targets + tile_w - 1) / tile_w;
  p.shift = shift;
  p.row_begin = row_begin; p.n_rows = n_rows; p.k = k;
  p.out_idx = out_idx; p.out_cnt = out_cnt; p.out_score = out_score;
  p.counter = static_cast<unsigned long long*>(ws);
  p.ablate = 0;
  if (const char* ab = std::getenv("DPATHSIM_ABLATE")) p.ablate = std::atoi(ab);
  DPS_HIP_RET(hipMemsetAsync(p.counter, 0, sizeof(unsigned long long), st));
  const size_t lds = hot_lds_bytes(shift);
  int dev = 0, n_cu = 256;
  DPS_HIP_RET(hipGetDevice(&dev));
  DPS_HIP_RET(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
  int per_cu = static_cast<int>((160 * 1024) / lds);
  if (per_cu < 1) per_cu = 1;
  if (per_cu > 16) per_cu = 16;
  int64_t grid = static_cast<int64_t>(n_cu) * per_cu;
  const int64_t need = (n_rows + kRowChunk - 1) / kRowChunk;
  if (grid > need) grid = need;
  if (k <= 64) return launch_hot<1>(p, lds, grid, st);
  if (k <= 128) return launch_hot<2>(p, lds, grid, st);
  return launch_hot<4>(p, lds, grid, st);
}

int dps_walk_row(const int32_t* src_col, const int32_t* src_val, int64_t src_len,
                 const int32_t* t_perm, int64_t n_targets, int64_t n_mids, int32_t tile_w,
                 const uint32_t* tile_off, const uint32_t* tile_ent, int64_t* out_m,
                 void* stream) {
  (void)n_mids;
  const int shift = log2_exact(tile_w);
  DPS_REQUIRE(shift >= 8 && shift <= 14, DPS_ERR_UNSUPPORTED, "bad tile_w %d", tile_w);
  DPS_REQUIRE(src_len >= 0 && n_targets >= 0, DPS_ERR_INVALID, "negative size");
  auto st = static_cast<hipStream_t>(stream);
  const int64_t T = (n_targets + tile_w - 1) / tile_w;
  if (T == 0) return DPS_OK;
  DPS_HIP_RET(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_walk_row),
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  static_cast<int>(tile_w * sizeof(int32_t))));
  k_walk_row<<<static_cast<unsigned>(T), kBlock, static_cast<size_t>(tile_w) * sizeof(int32_t),
               st>>>(src_col, src_val, src_len, n_targets, shift, T, tile_off, tile_ent, t_perm,
                     out_m);
  DPS_LAUNCHED();
  return DPS_OK;
}

int dps_row_scores(const int64_t* m, const int64_t* g, int64_t gx, int64_t n, double* score,
                   int64_t* zero_div, void* stream) {
  DPS_REQUIRE(n >= 0 && gx >= 0, DPS_ERR_INVALID, "bad arguments");
  auto st = static_cast<hipStream_t>(stream);
  if (zero_div) DPS_HIP_RET(hipMemsetAsync(zero_div, 0, sizeof(int64_t), st));
  if (n == 0) return DPS_OK;
  k_row_scores<<<grid_for(n, kBlock), kBlock, 0, st>>>(
      m, g, gx, n, score, reinterpret_cast<unsigned long long*>(zero_div));
  DPS_LAUNCHED();
  return DPS_OK;
}

int dps_pair_count(const int32_t* a_col, const int32_t* a_val, int64_t a_len,
                   const int32_t* b_col, const int32_t* b_val, int64_t b_len, int64_t* out,
                   void* stream) {
  DPS_REQUIRE(a_len >= 0 && b_len >= 0 && out, DPS_ERR_INVALID, "bad arguments");
  auto st = static_cast<hipStream_t>(stream);
  k_pair_count<<<1, kWave, 0, st>>>(a_col, a_val, a_len, b_col, b_val, b_len, out);
  DPS_LAUNCHED();
  return DPS_OK;
}

}  // extern "C"
