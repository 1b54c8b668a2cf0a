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

namespace dps {
namespace {

constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kRowChunk = 4;  // rows per dequeue

// --------------------------------------------------------------------------
// Tile build: counting sort of C entries into (v, t) buckets.
__global__ __launch_bounds__(kBlock) void k_tile_count(const int64_t* __restrict__ c_ptr,
                                                       const int32_t* __restrict__ c_col,
                                                       const int32_t* __restrict__ c_val,
                                                       int64_t n_rows, int shift, int64_t T,
                                                       uint32_t* __restrict__ cnt,
                                                       int32_t* __restrict__ status) {
  const int lane = lane_id();
  const int64_t wave0 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWavesPerBlock;
  for (int64_t y = wave0; y < n_rows; y += nwaves) {
    const int64_t t = y >> shift;
    for (int64_t j = c_ptr[y] + lane; j < c_ptr[y + 1]; j += kWave) {
      if (c_val[j] > 0xFFFF && status) *status = DPS_ERR_OVERFLOW;
      atomicAdd(&cnt[static_cast<int64_t>(c_col[j]) * T + t], 1u);
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
                                                         int64_t n_rows, int shift, int64_t T,
                                                         const int64_t* __restrict__ off,
                                                         uint32_t* __restrict__ cursor,
                                                         uint32_t* __restrict__ ent) {
  const int lane = lane_id();
  const int64_t wave0 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWavesPerBlock;
  const uint32_t ymask = (1u << shift) - 1u;
  for (int64_t y = wave0; y < n_rows; y += nwaves) {
    const int64_t t = y >> shift;
    for (int64_t j = c_ptr[y] + lane; j < c_ptr[y + 1]; j += kWave) {
      const int64_t b = static_cast<int64_t>(c_col[j]) * T + t;
      const uint32_t pos = atomicAdd(&cursor[b], 1u);
      ent[off[b] + pos] =
          (static_cast<uint32_t>(c_val[j]) << 16) | (static_cast<uint32_t>(y) & ymask);
    }
  }
}

// --------------------------------------------------------------------------
// Top-k helpers.  Order: score desc, then target index asc.
__device__ __forceinline__ bool better(double s1, int y1, double s2, int y2) {
  return s1 > s2 || (s1 == s2 && y1 < y2);
}

// Smallest m >= 0 with fl(2m / (gx + m)) >= kth.  Since g[y] >= M[x,y] for
// every target (g[y] sums M[y,.] over all rows, x included), fl(2M/(gx+gy))
// <= fl(2M/(gx+M)) and the map m -> 2m/(gx+m) is increasing: any candidate
// with M < mmin scores strictly below the current k-th and is rejected with
// one integer compare (no g load, no division).
__device__ int compute_mmin(double kth, int64_t gx) {
  if (kth <= 0.0 || gx <= 0) return 0;
  double est = kth * static_cast<double>(gx) / (2.0 - kth);
  int64_t m = static_cast<int64_t>(est) - 2;
  if (m < 0) m = 0;
  while (static_cast<double>(2 * m) / static_cast<double>(gx + m) < kth) ++m;
  while (m > 0 && static_cast<double>(2 * (m - 1)) / static_cast<double>(gx + m - 1) >= kth) --m;
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
  const int64_t* g;
  const uint32_t* tile_off;
  const uint32_t* tile_ent;
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
};

// Per-wave LDS image: acc int32[W] | bitmap uint32[W/32] | list uint16[W].
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int KPL>
__global__ __launch_bounds__(kWave) void k_cct_topk(HotParams p) {
  extern __shared__ __attribute__((aligned(16))) int32_t lds[];
  const int lane = threadIdx.x;
  const int W = 1 << p.shift;
  const int nwords = W >> 5;
  int32_t* acc = lds;
  uint32_t* bitmap = reinterpret_cast<uint32_t*>(lds + W);
  uint16_t* list = reinterpret_cast<uint16_t*>(lds + W + nwords);

  for (int i = lane; i < W; i += kWave) acc[i] = 0;
  for (int i = lane; i < nwords; i += kWave) bitmap[i] = 0;
  wave_lds_fence();

  for (;;) {
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(p.counter, static_cast<unsigned long long>(kRowChunk));
    base = __shfl(base, 0, kWave);
    if (static_cast<int64_t>(base) >= p.n_rows) break;
    const int64_t r_end = min(static_cast<int64_t>(base) + kRowChunk, p.n_rows);
    for (int64_t r = static_cast<int64_t>(base); r < r_end; ++r) {
      const int64_t x = p.row_begin + r;
      const int64_t pb = p.c_ptr[x];
      const int d = static_cast<int>(p.c_ptr[x + 1] - pb);
      const int64_t gx = p.g[x];
      TopK<KPL> top;
      top.init(p.k);
      int mmin = 0;

      // Row venues: the fast path keeps them in registers (d <= 64).
      int v_reg = 0, c_reg = 0;
      uint32_t lo_reg = 0, hi_reg = 0;
      if (d <= kWave && lane < d) {
        v_reg = p.c_col[pb + lane];
        c_reg = p.c_val[pb + lane];
        const int64_t vb = static_cast<int64_t>(v_reg) * p.T;
        lo_reg = p.tile_off[vb];
        hi_reg = p.tile_off[vb + 1];
      }
      for (int64_t t = 0; t < p.T; ++t) {
        // ---- scatter --------------------------------------------------------
        uint32_t scattered = 0;
        if (d <= kWave) {
          // prefetch the next tile's bucket end while this tile runs
          uint32_t hi_next = 0;
          if (lane < d && t + 1 < p.T) hi_next = p.tile_off[static_cast<int64_t>(v_reg) * p.T + t + 2];
          for (int jj = 0; jj < d; ++jj) {
            const uint32_t l = readlane(lo_reg, jj), h = readlane(hi_reg, jj);
            if (l == h) continue;
            const int cj = readlane(c_reg, jj);
            scattered += h - l;
            for (uint32_t i = l + lane; i < h; i += kWave) {
              const uint32_t e = p.tile_ent[i];
              const int yl = static_cast<int>(e & 0xFFFFu);
              atomicAdd(&acc[yl], cj * static_cast<int>(e >> 16));
              atomicOr(&bitmap[yl >> 5], 1u << (yl & 31));
            }
          }
          lo_reg = hi_reg;
          hi_reg = hi_next;
        } else {
          for (int c0 = 0; c0 < d; c0 += kWave) {
            const int j = c0 + lane;
            int cx = 0;
            uint32_t lo = 0, hi = 0;
            if (j < d) {
              const int64_t vb = static_cast<int64_t>(p.c_col[pb + j]) * p.T + t;
              cx = p.c_val[pb + j];
              lo = p.tile_off[vb];
              hi = p.tile_off[vb + 1];
            }
            const int nj = min(kWave, d - c0);
            for (int jj = 0; jj < nj; ++jj) {
              const uint32_t l = readlane(lo, jj), h = readlane(hi, jj);
              if (l == h) continue;
              const int cj = readlane(cx, jj);
              scattered += h - l;
              for (uint32_t i = l + lane; i < h; i += kWave) {
                const uint32_t e = p.tile_ent[i];
                const int yl = static_cast<int>(e & 0xFFFFu);
                atomicAdd(&acc[yl], cj * static_cast<int>(e >> 16));
                atomicOr(&bitmap[yl >> 5], 1u << (yl & 31));
              }
            }
          }
        }
        if (scattered == 0) continue;
        wave_lds_fence();
        // ---- compact bitmap -> touched list --------------------------------
        int n_list = 0;
        for (int w0 = 0; w0 < nwords; w0 += kWave) {
          const int w = w0 + lane;
          uint32_t bits = 0;
          if (w < nwords) {
            bits = bitmap[w];
            if (bits) bitmap[w] = 0;
          }
          const int pc = __popc(bits);
          const int inc = wave_inclusive_sum(pc);
          int o = n_list + inc - pc;
          while (bits) {
            const int b = __ffs(bits) - 1;
            bits &= bits - 1;
            list[o++] = static_cast<uint16_t>((w << 5) | b);
          }
          n_list += readlane(inc, kWave - 1);
        }
        wave_lds_fence();
        // ---- epilogue: exact score + top-k ---------------------------------
        const int64_t y0 = t << p.shift;
        const double kth_before = top.kth_s;
        for (int i0 = 0; i0 < n_list; i0 += kWave) {
          const int i = i0 + lane;
          int yl = 0, M = 0;
          if (i < n_list) {
            yl = list[i];
            M = acc[yl];
            acc[yl] = 0;
          }
          const int y = static_cast<int>(y0 + yl);
          bool cand = (i < n_list) && (y != x) && (M >= mmin);
          double sc = 0.0;
          if (cand) {
            const int64_t den = gx + p.g[y];
            sc = den ? static_cast<double>(2 * static_cast<int64_t>(M)) / static_cast<double>(den)
                     : 0.0;
            cand = better(sc, y, top.kth_s, top.kth_y);
          }
          uint64_t mask = ballot(cand);
          while (mask) {
            const int src = __ffsll(static_cast<long long>(mask)) - 1;
            mask &= mask - 1;
            const double cs = readlane(sc, src);
            const int cy = readlane(y, src);
            if (!better(cs, cy, top.kth_s, top.kth_y)) continue;
            top.insert(cs, cy, readlane(M, src));
          }
        }
        if (top.filled == top.k && top.kth_s != kth_before) mmin = compute_mmin(top.kth_s, gx);
        wave_lds_fence();
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
        // exclude targets already ranked (wave-uniform loop over the ranked set)
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
// Single-source dense row: one block per target tile.
__global__ __launch_bounds__(kBlock) void k_walk_row(const int32_t* __restrict__ src_col,
                                                     const int32_t* __restrict__ src_val,
                                                     int64_t src_len, int64_t n_targets, int shift,
                                                     int64_t T, const uint32_t* __restrict__ off,
                                                     const uint32_t* __restrict__ ent,
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
  for (int i = threadIdx.x; i < W && y0 + i < n_targets; i += kBlock) out_m[y0 + i] = acc[i];
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
  while ((1 << s) < w) ++s;
  return (1 << s) == w ? s : -1;
}

}  // namespace
}  // namespace dps

using namespace dps;

extern "C" {

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
                       int64_t n_targets, int64_t n_mids, int32_t tile_w, uint32_t* tile_off,
                       uint32_t* tile_ent, int32_t* status_dev, void* ws, size_t ws_bytes,
                       void* stream) {
  const int shift = log2_exact(tile_w);
  DPS_REQUIRE(shift >= 8 && shift <= 14, DPS_ERR_UNSUPPORTED,
              "tile_w must be a power of two in [256, 16384], got %d", tile_w);
  DPS_REQUIRE(n_targets >= 0 && n_mids >= 0, DPS_ERR_INVALID, "negative size");
  DPS_REQUIRE(n_targets < INT32_MAX, DPS_ERR_OVERFLOW, "n_targets exceeds int32");
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
  if (n_targets > 0 && nb > 0) {
    k_tile_count<<<grid_for(n_targets * kWave, kBlock), kBlock, 0, st>>>(
        c_ptr, c_col, c_val, n_targets, shift, T, cnt, status_dev);
    DPS_LAUNCHED();
  }
  DPS_HIP_RET(scan_exclusive<uint32_t>(cnt, off64, nb, sws, scan_ws, st));
  k_tile_off32<<<grid_for(nb + 1, kBlock), kBlock, 0, st>>>(off64, nb, tile_off);
  DPS_LAUNCHED();
  if (n_targets > 0 && nb > 0) {
    k_tile_scatter<<<grid_for(n_targets * kWave, kBlock), kBlock, 0, st>>>(
        c_ptr, c_col, c_val, n_targets, shift, T, off64, cursor, tile_ent);
    DPS_LAUNCHED();
  }
  return DPS_OK;
}

size_t dps_cct_topk_workspace_size(void) { return 256; }

static size_t hot_lds_bytes(int shift) {
  const size_t W = size_t(1) << shift;
  return W * sizeof(int32_t) + (W / 32) * sizeof(uint32_t) + W * sizeof(uint16_t);
}

int dps_cct_topk(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                 const int64_t* g, int64_t n_targets, int64_t n_mids, int32_t tile_w,
                 const uint32_t* tile_off, const uint32_t* tile_ent, int64_t row_begin,
                 int64_t row_end, int32_t k, int32_t* out_idx, int64_t* out_cnt,
                 double* out_score, void* ws, size_t ws_bytes, void* stream) {
  (void)n_mids;
  const int shift = log2_exact(tile_w);
  DPS_REQUIRE(shift >= 8 && shift <= 14, DPS_ERR_UNSUPPORTED,
              "tile_w must be a power of two in [256, 16384], got %d", tile_w);
  DPS_REQUIRE(k >= 1 && k <= 256, DPS_ERR_UNSUPPORTED, "k must be in [1, 256], got %d", k);
  DPS_REQUIRE(0 <= row_begin && row_begin <= row_end && row_end <= n_targets, DPS_ERR_INVALID,
              "row range [%lld, %lld) outside [0, %lld)", static_cast<long long>(row_begin),
              static_cast<long long>(row_end), static_cast<long long>(n_targets));
  DPS_REQUIRE(n_targets < INT32_MAX, DPS_ERR_OVERFLOW, "n_targets exceeds int32");
  DPS_REQUIRE(ws && ws_bytes >= dps_cct_topk_workspace_size(), DPS_ERR_WORKSPACE,
              "cct_topk workspace too small");
  auto st = static_cast<hipStream_t>(stream);
  const int64_t n_rows = row_end - row_begin;
  if (n_rows == 0) return DPS_OK;
  HotParams p;
  p.c_ptr = c_ptr; p.c_col = c_col; p.c_val = c_val; p.g = g;
  p.tile_off = tile_off; p.tile_ent = tile_ent;
  p.n_targets = n_targets;
  p.T = (n_targets + tile_w - 1) / tile_w;
  p.shift = shift;
  p.row_begin = row_begin; p.n_rows = n_rows; p.k = k;
  p.out_idx = out_idx; p.out_cnt = out_cnt; p.out_score = out_score;
  p.counter = static_cast<unsigned long long*>(ws);
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
  if (k <= 64) {
    DPS_HIP_RET(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_cct_topk<1>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize,
                                    static_cast<int>(lds)));
    k_cct_topk<1><<<static_cast<unsigned>(grid), kWave, lds, st>>>(p);
  } else if (k <= 128) {
    DPS_HIP_RET(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_cct_topk<2>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize,
                                    static_cast<int>(lds)));
    k_cct_topk<2><<<static_cast<unsigned>(grid), kWave, lds, st>>>(p);
  } else {
    DPS_HIP_RET(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_cct_topk<4>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize,
                                    static_cast<int>(lds)));
    k_cct_topk<4><<<static_cast<unsigned>(grid), kWave, lds, st>>>(p);
  }
  DPS_LAUNCHED();
  return DPS_OK;
}

int dps_walk_row(const int32_t* src_col, const int32_t* src_val, int64_t src_len,
                 int64_t n_targets, int64_t n_mids, int32_t tile_w, const uint32_t* tile_off,
                 const uint32_t* tile_ent, int64_t* out_m, void* stream) {
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
               st>>>(src_col, src_val, src_len, n_targets, shift, T, tile_off, tile_ent, out_m);
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
