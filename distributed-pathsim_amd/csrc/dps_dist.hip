// Multi-GPU row sharding helpers, so that an N-GPU step runs
// no PyTorch compute between its first and last event:
//   dps_shard_edges     work-balanced contiguous row shards from the build's
//                       per-row work terms (device scan + binary search), and
//                       the comparison with a reference plan (no read-back);
//   dps_pack_counts     (count << 32) | index words of a top-k block, the
//                       8-byte wire format of the gather;
//   dps_unpack_gathered rank 0's gathered [world * m, k] words back to
//                       (index, count, score) in row order, the score rebuilt
//                       with the hot kernel's one fp64 division of the same
//                       exact integers (DPathSim_APVPA.py:51-52), so the bits
//                       are identical to the ones the rank computed.
//   dps_label_rows      the rows of C of a target-label range, in label order:
//                       the input of one rank's slice of the C^T tile build;
//   dps_tiles_pack      a slice build's offsets, maxima, tile minima and
//                       entries packed into one fixed-size buffer (the unit of
//                       the all-gather), with an overflow flag;
//   dps_tiles_assemble  the full [v][t] tile layout from every rank's slice,
//                       rebased: one scan over (venue, rank) runs, one copy.
// The reference has no counterpart: its Spark session (:146-168) moves the
// .count() results (:86, :107) back to the driver one target at a time, and
// every executor re-joins the whole graph (:72-76).
#include <algorithm>

#include "dps_common.hpp"

namespace dps {
namespace {

constexpr int kBlock = 256;

// edges[r] (r = 1..world-1) = number of rows i whose inclusive work prefix
// W(i) = pre[i+1] + (i+1) * hm is <= cut_r = r * W(n-1) / world, with
// hm = (sum terms / n) / 2 -- the row work terms + half the mean of
// PathSimEngine.row_work().  W is nondecreasing, so a binary search per cut.
__global__ __launch_bounds__(kBlock) void k_shard_edges(const int64_t* __restrict__ pre, int64_t n,
                                                        int world, int64_t* __restrict__ edges,
                                                        const int64_t* __restrict__ ref,
                                                        int64_t* __restrict__ mismatch) {
  __shared__ int64_t e[kBlock + 1];
  const int r = threadIdx.x;
  const int64_t S = pre[n];
  const int64_t hm = (S / n) / 2;
  const int64_t total = S + n * hm;
  if (r <= world) {
    int64_t v;
    if (r == 0) {
      v = 0;
    } else if (r == world) {
      v = n;
    } else {
      const int64_t cut = static_cast<int64_t>(r) * total / world;
      int64_t lo = 0, hi = n;                     // count of i with W(i) <= cut
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (pre[mid + 1] + (mid + 1) * hm <= cut) lo = mid + 1;
        else hi = mid;
      }
      v = lo;
    }
    e[r] = v;
  }
  __syncthreads();
  if (r == 0) {                                    // running maximum (monotone already)
    int64_t m = 0, bad = 0;
    for (int i = 0; i <= world; ++i) {
      m = e[i] > m ? e[i] : m;
      m = m < n ? m : n;
      edges[i] = m;
      if (ref) bad += ref[i] != m;
    }
    if (ref && mismatch) *mismatch += bad;
  }
}

__global__ __launch_bounds__(kBlock) void k_shard_edges_empty(int world, int64_t* __restrict__ edges,
                                                              const int64_t* __restrict__ ref,
                                                              int64_t* __restrict__ mismatch) {
  if (threadIdx.x != 0) return;
  int64_t bad = 0;
  for (int i = 0; i <= world; ++i) {
    edges[i] = 0;
    if (ref) bad += ref[i] != 0;
  }
  if (ref && mismatch) *mismatch += bad;
}

__global__ __launch_bounds__(kBlock) void k_pack_counts(const int32_t* __restrict__ idx,
                                                        const int64_t* __restrict__ cnt, int64_t n,
                                                        int64_t* __restrict__ out) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * kBlock)
    out[i] = static_cast<int64_t>((static_cast<uint64_t>(cnt[i]) << 32) |
                                  static_cast<uint32_t>(idx[i]));
}

// One thread per output slot: row x = edges[0] + i / k lives in the shard r
// with edges[r] <= x < edges[r+1], at gathered row r * m + (x - edges[r]).
__global__ __launch_bounds__(kBlock) void k_unpack_gathered(const int64_t* __restrict__ gathered,
                                                            int world, int64_t m, int k,
                                                            int64_t n_rows,
                                                            const int64_t* __restrict__ edges,
                                                            const int64_t* __restrict__ den,
                                                            int32_t* __restrict__ out_idx,
                                                            int64_t* __restrict__ out_cnt,
                                                            double* __restrict__ out_score) {
  const int64_t x0 = edges[0];
  // the out_* arrays hold n_rows rows: never more, whatever the device edges say
  const int64_t span = edges[world] - x0;
  const int64_t n = (span < n_rows ? span : n_rows) * k;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * kBlock) {
    const int64_t x = x0 + i / k;
    const int s = static_cast<int>(i % k);
    int r = 0;
    while (r + 1 < world && edges[r + 1] <= x) ++r;
    if (x - edges[r] >= m) continue;   // a shard longer than the gathered block: not sent
    const uint64_t w = static_cast<uint64_t>(gathered[(r * m + (x - edges[r])) * k + s]);
    const int32_t y = static_cast<int32_t>(static_cast<uint32_t>(w));
    const int64_t c = static_cast<int64_t>(w >> 32);
    double sc = 0.0;
    if (y >= 0 && c > 0)
      sc = static_cast<double>(2 * c) / static_cast<double>(den[x] + den[y]);
    out_idx[i] = y;
    out_cnt[i] = c;
    out_score[i] = sc;
  }
}

// ---- tile-range slices of the C^T build (N > 1) ------------------------------
// Sub-C row i = C row t_perm[l0 + i]: its length, then (after a scan) its entries.
__global__ __launch_bounds__(kBlock) void k_label_row_len(const int64_t* __restrict__ c_ptr,
                                                          const int32_t* __restrict__ t_perm,
                                                          int64_t l0, int64_t n,
                                                          int64_t* __restrict__ len) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * kBlock) {
    const int64_t y = t_perm ? t_perm[l0 + i] : l0 + i;
    len[i] = c_ptr[y + 1] - c_ptr[y];
  }
}

// One wave per 64 sub-rows; each row's entries copied by the whole wave
// (rows are short: ~7 entries on config3, ~30 on config4).
__global__ __launch_bounds__(kBlock) void k_label_row_copy(const int64_t* __restrict__ c_ptr,
                                                           const int32_t* __restrict__ c_col,
                                                           const int32_t* __restrict__ c_val,
                                                           const int32_t* __restrict__ t_perm,
                                                           int64_t l0, int64_t n,
                                                           const int64_t* __restrict__ sub_ptr,
                                                           int32_t* __restrict__ sub_col,
                                                           int32_t* __restrict__ sub_val) {
  const int lane = lane_id();
  const int64_t wave0 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * (kBlock / kWave);
  for (int64_t i = wave0; i < n; i += nwaves) {
    const int64_t y = t_perm ? t_perm[l0 + i] : l0 + i;
    const int64_t b = c_ptr[y], e = c_ptr[y + 1], o = sub_ptr[i];
    for (int64_t j = lane; j < e - b; j += kWave) {
      sub_col[o + j] = c_col[b + j];
      sub_val[o + j] = c_val[b + j];
    }
  }
}

// Slice layout (uint32 words, fixed per (n_mids, Tr, cap)): off[n_mids*Tr+1],
// maxc[n_mids*Tr+1], then gmin (int64[Tr], 8-byte aligned), then ent[cap]
// (16-byte aligned; cap a multiple of 4, so every slice starts 16-byte aligned);
// the slice's own tiles Tl <= Tr use stride Tl in off / maxc ([v][tl]).
struct SliceLayout {
  int64_t nb1, off, maxc, gmin, ent, words;
  __host__ __device__ SliceLayout(int64_t n_mids, int64_t Tr, int64_t cap) {
    nb1 = n_mids * Tr + 1;
    off = 0;
    maxc = nb1;
    gmin = (2 * nb1 + 1) & ~int64_t(1);
    ent = (gmin + 2 * Tr + 3) & ~int64_t(3);      // 16-byte aligned (uint4 copies)
    words = ent + cap;                             // cap is a multiple of 4 words

  }
};

__global__ __launch_bounds__(kBlock) void k_tiles_pack(const uint32_t* __restrict__ off,
                                                       const uint32_t* __restrict__ maxc,
                                                       const int64_t* __restrict__ gmin,
                                                       const uint32_t* __restrict__ ent,
                                                       int64_t n_mids, int64_t Tl, int64_t Tr,
                                                       int64_t cap, uint32_t* __restrict__ slice,
                                                       int32_t* __restrict__ overflow) {
  const SliceLayout L(n_mids, Tr, cap);
  const int64_t nbl = n_mids * Tl;
  const int64_t words = nbl > 0 ? static_cast<int64_t>(off[nbl]) : 0;
  if (blockIdx.x == 0 && threadIdx.x == 0 && words > cap && overflow) *overflow = DPS_ERR_OVERFLOW;
  const int64_t nw = words < cap ? words : cap;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  const int64_t t0 = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  for (int64_t i = t0; i <= nbl; i += stride) {
    slice[L.off + i] = nbl > 0 ? off[i] : 0u;
    slice[L.maxc + i] = nbl > 0 && maxc ? maxc[i] : 0u;
  }
  int64_t* g = reinterpret_cast<int64_t*>(slice + L.gmin);
  for (int64_t i = t0; i < Tl; i += stride) g[i] = gmin ? gmin[i] : 0;
  const uint4* src = reinterpret_cast<const uint4*>(ent);
  uint4* dst = reinterpret_cast<uint4*>(slice + L.ent);   // bucket runs are 16-byte multiples
  for (int64_t i = t0; i < nw / 4; i += stride) dst[i] = src[i];
}

// Tiles of rank r: [r*Tr, r*Tr + Tl_r), Tl_r = clamp(T - r*Tr, 0, Tr).
__device__ __forceinline__ int64_t slice_tiles(int64_t T, int64_t Tr, int r) {
  const int64_t t = T - static_cast<int64_t>(r) * Tr;
  return t < 0 ? 0 : t < Tr ? t : Tr;
}

// Run (v, r): venue v's buckets of rank r's tiles, contiguous in both layouts.
// A slice whose offsets leave its entry capacity (a failed collective, a
// plan that no longer fits) sets *status; the layout is then left empty.
__global__ __launch_bounds__(kBlock) void k_tiles_runs(const uint32_t* __restrict__ gathered,
                                                       int64_t slice_words, int world,
                                                       int64_t n_mids, int64_t T, int64_t Tr,
                                                       int64_t cap, int64_t* __restrict__ run,
                                                       int32_t* __restrict__ status) {
  const SliceLayout L(n_mids, Tr, cap);
  const int64_t n = n_mids * world;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * kBlock) {
    const int64_t v = i / world;
    const int r = static_cast<int>(i - v * world);
    const int64_t Tl = slice_tiles(T, Tr, r);
    const uint32_t* off = gathered + r * slice_words + L.off;
    int64_t len = 0;
    if (Tl > 0) {
      const int64_t a = off[v * Tl], b = off[(v + 1) * Tl];
      if (a > b || b > cap || (a & 3) != 0) {
        *status = DPS_ERR_OVERFLOW;
      } else {
        len = b - a;
      }
    }
    run[i] = len;
  }
}

__global__ __launch_bounds__(kBlock) void k_tiles_offsets(const uint32_t* __restrict__ gathered,
                                                          int64_t slice_words, int world,
                                                          int64_t n_mids, int64_t T, int64_t Tr,
                                                          int64_t cap,
                                                          const int64_t* __restrict__ base,
                                                          int64_t ent_words,
                                                          const int32_t* __restrict__ status,
                                                          uint32_t* __restrict__ tile_off,
                                                          uint32_t* __restrict__ tile_maxc,
                                                          int64_t* __restrict__ tile_gmin) {
  const SliceLayout L(n_mids, Tr, cap);
  const int64_t nb = n_mids * T;
  // a bad slice (or a layout beyond tile_ent's capacity): every bucket empty
  const bool bad = *status != 0 || base[n_mids * world] > ent_words;
  for (int64_t b = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; b <= nb;
       b += static_cast<int64_t>(gridDim.x) * kBlock) {
    if (b == nb) {
      tile_off[nb] = bad ? 0u : static_cast<uint32_t>(base[n_mids * world]);
      if (tile_maxc) tile_maxc[nb] = 0u;
      continue;
    }
    if (bad) {
      tile_off[b] = 0u;
      if (tile_maxc) tile_maxc[b] = 0u;
      if (tile_gmin && b < T) tile_gmin[b] = 0;
      continue;
    }
    const int64_t v = b / T, t = b - v * T;
    const int r = static_cast<int>(t / Tr);
    const int64_t tl = t - r * Tr, Tl = slice_tiles(T, Tr, r);
    const uint32_t* sl = gathered + r * slice_words;
    const uint32_t* off = sl + L.off;
    // inside the run (checked by k_tiles_runs), so inside tile_ent
    int64_t o = static_cast<int64_t>(off[v * Tl + tl]) - off[v * Tl];
    const int64_t len = base[v * world + r + 1] - base[v * world + r];
    o = o < 0 ? 0 : o > len ? len : o;
    tile_off[b] = static_cast<uint32_t>(base[v * world + r] + o);
    if (tile_maxc) tile_maxc[b] = sl[L.maxc + v * Tl + tl];
    if (tile_gmin && v == 0) tile_gmin[t] = reinterpret_cast<const int64_t*>(sl + L.gmin)[tl];
  }
}

// One wave per run: 16-byte words from the slice's entries to the full layout.
__global__ __launch_bounds__(kBlock) void k_tiles_copy(const uint32_t* __restrict__ gathered,
                                                       int64_t slice_words, int world,
                                                       int64_t n_mids, int64_t T, int64_t Tr,
                                                       int64_t cap, const int64_t* __restrict__ base,
                                                       int64_t ent_words,
                                                       const int32_t* __restrict__ status,
                                                       uint32_t* __restrict__ tile_ent) {
  const SliceLayout L(n_mids, Tr, cap);
  if (*status != 0 || base[n_mids * world] > ent_words) return;
  const int lane = lane_id();
  const int64_t n = n_mids * world;
  const int64_t wave0 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * (kBlock / kWave);
  for (int64_t i = wave0; i < n; i += nwaves) {
    const int64_t v = i / world;
    const int r = static_cast<int>(i - v * world);
    const int64_t Tl = slice_tiles(T, Tr, r);
    if (Tl == 0) continue;
    const uint32_t* sl = gathered + r * slice_words;
    const int64_t s0 = sl[L.off + v * Tl];
    const int64_t len = base[i + 1] - base[i];
    const uint4* src = reinterpret_cast<const uint4*>(sl + L.ent + s0);
    uint4* dst = reinterpret_cast<uint4*>(tile_ent + base[i]);
    for (int64_t j = lane; j < len / 4; j += kWave) dst[j] = src[j];
  }
}

}  // namespace
}  // namespace dps

using namespace dps;

extern "C" {

size_t dps_shard_edges_workspace_size(int64_t n_rows) {
  if (n_rows < 0) return 0;
  return align_up(static_cast<size_t>(n_rows + 1) * sizeof(int64_t)) + scan_workspace_size(n_rows) +
         256;
}

int dps_shard_edges(const int64_t* terms, int64_t n_rows, int32_t world, int64_t* edges,
                    const int64_t* edges_ref, int64_t* mismatch, void* ws, size_t ws_bytes,
                    void* stream) {
  DPS_REQUIRE(world >= 1 && world <= kBlock - 1, DPS_ERR_INVALID, "world must be in [1, %d], got %d",
              kBlock - 1, world);
  DPS_REQUIRE(n_rows >= 0, DPS_ERR_INVALID, "bad n_rows");
  DPS_REQUIRE(edges, DPS_ERR_INVALID, "null edges");
  DPS_REQUIRE(!edges_ref || mismatch, DPS_ERR_INVALID, "edges_ref needs a mismatch counter");
  auto st = static_cast<hipStream_t>(stream);
  if (n_rows == 0) {
    k_shard_edges_empty<<<1, kBlock, 0, st>>>(world, edges, edges_ref, mismatch);
    DPS_LAUNCHED();
    return DPS_OK;
  }
  DPS_REQUIRE(terms, DPS_ERR_INVALID, "null terms");
  Carve cv(ws, ws_bytes);
  int64_t* pre = cv.take<int64_t>(static_cast<size_t>(n_rows + 1));
  const size_t sb = scan_workspace_size(n_rows);
  void* sws = cv.take<char>(sb);
  DPS_REQUIRE(cv.ok, DPS_ERR_WORKSPACE, "workspace too small (%zu bytes)", ws_bytes);
  DPS_HIP_RET(scan_exclusive<int64_t>(terms, pre, n_rows, sws, sb, st));
  k_shard_edges<<<1, kBlock, 0, st>>>(pre, n_rows, world, edges, edges_ref, mismatch);
  DPS_LAUNCHED();
  return DPS_OK;
}

int dps_pack_counts(const int32_t* idx, const int64_t* cnt, int64_t n, int64_t* out, void* stream) {
  DPS_REQUIRE(n >= 0, DPS_ERR_INVALID, "bad n");
  if (n == 0) return DPS_OK;
  DPS_REQUIRE(idx && cnt && out, DPS_ERR_INVALID, "null array");
  k_pack_counts<<<grid_for(n, kBlock), kBlock, 0, static_cast<hipStream_t>(stream)>>>(idx, cnt, n, out);
  DPS_LAUNCHED();
  return DPS_OK;
}

int dps_unpack_gathered(const int64_t* gathered, int32_t world, int64_t m, int32_t k,
                        const int64_t* edges, int64_t n_rows, const int64_t* den, int32_t* out_idx,
                        int64_t* out_cnt, double* out_score, void* stream) {
  DPS_REQUIRE(world >= 1, DPS_ERR_INVALID, "bad world %d", world);
  DPS_REQUIRE(k >= 1 && m >= 0 && n_rows >= 0, DPS_ERR_INVALID, "bad k / m / n_rows");
  if (n_rows == 0) return DPS_OK;
  DPS_REQUIRE(gathered && edges && den && out_idx && out_cnt && out_score, DPS_ERR_INVALID,
              "null array");
  k_unpack_gathered<<<grid_for(n_rows * k, kBlock), kBlock, 0, static_cast<hipStream_t>(stream)>>>(
      gathered, world, m, k, n_rows, edges, den, out_idx, out_cnt, out_score);
  DPS_LAUNCHED();
  return DPS_OK;
}

// ---- tile-range slices of the C^T build (N > 1) ------------------------------
size_t dps_label_rows_workspace_size(int64_t n) {
  if (n < 0) return 0;
  return align_up(static_cast<size_t>(n + 1) * sizeof(int64_t)) + scan_workspace_size(n) + 256;
}

int dps_label_rows(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                   const int32_t* t_perm, int64_t l0, int64_t l1, int64_t* sub_ptr,
                   int32_t* sub_col, int32_t* sub_val, void* ws, size_t ws_bytes, void* stream) {
  DPS_REQUIRE(l0 >= 0 && l1 >= l0, DPS_ERR_INVALID, "bad label range [%lld, %lld)",
              static_cast<long long>(l0), static_cast<long long>(l1));
  DPS_REQUIRE(c_ptr && sub_ptr, DPS_ERR_INVALID, "null array");
  auto st = static_cast<hipStream_t>(stream);
  const int64_t n = l1 - l0;
  if (n == 0) {
    DPS_HIP_RET(hipMemsetAsync(sub_ptr, 0, sizeof(int64_t), st));
    return DPS_OK;
  }
  DPS_REQUIRE(c_col && c_val && sub_col && sub_val, DPS_ERR_INVALID, "null array");
  Carve cv(ws, ws_bytes);
  int64_t* len = cv.take<int64_t>(static_cast<size_t>(n + 1));
  const size_t sb = scan_workspace_size(n);
  void* sws = cv.take<char>(sb);
  DPS_REQUIRE(cv.ok, DPS_ERR_WORKSPACE, "workspace too small (%zu bytes)", ws_bytes);
  k_label_row_len<<<grid_for(n, kBlock), kBlock, 0, st>>>(c_ptr, t_perm, l0, n, len);
  DPS_LAUNCHED();
  DPS_HIP_RET(scan_exclusive<int64_t>(len, sub_ptr, n, sws, sb, st));
  k_label_row_copy<<<grid_for(n * kWave, kBlock, 4096), kBlock, 0, st>>>(
      c_ptr, c_col, c_val, t_perm, l0, n, sub_ptr, sub_col, sub_val);
  DPS_LAUNCHED();
  return DPS_OK;
}

int64_t dps_tiles_slice_words(int64_t n_mids, int64_t tiles_per_rank, int64_t ent_cap) {
  if (n_mids < 0 || tiles_per_rank < 0 || ent_cap < 0) return 0;
  return SliceLayout(n_mids, tiles_per_rank, (ent_cap + 3) / 4 * 4).words;
}

int dps_tiles_pack(const uint32_t* tile_off, const uint32_t* tile_maxc, const int64_t* tile_gmin,
                   const uint32_t* tile_ent, int64_t n_mids, int64_t n_tiles,
                   int64_t tiles_per_rank, int64_t ent_cap, uint32_t* slice, int32_t* overflow,
                   void* stream) {
  DPS_REQUIRE(n_mids >= 0 && n_tiles >= 0 && n_tiles <= tiles_per_rank && ent_cap >= 0,
              DPS_ERR_INVALID, "bad slice shape");
  DPS_REQUIRE(slice && (n_tiles == 0 || (tile_off && tile_ent)), DPS_ERR_INVALID, "null array");
  const int64_t cap = (ent_cap + 3) / 4 * 4;
  const SliceLayout L(n_mids, tiles_per_rank, cap);
  const int64_t n = std::max<int64_t>(L.nb1, cap / 4);
  k_tiles_pack<<<grid_for(n, kBlock), kBlock, 0, static_cast<hipStream_t>(stream)>>>(
      tile_off, tile_maxc, tile_gmin, tile_ent, n_mids, n_tiles, tiles_per_rank, cap, slice,
      overflow);
  DPS_LAUNCHED();
  return DPS_OK;
}

size_t dps_tiles_assemble_workspace_size(int64_t n_mids, int32_t world) {
  if (n_mids < 0 || world < 1) return 0;
  const int64_t n = n_mids * world;
  return 2 * align_up(static_cast<size_t>(n + 1) * sizeof(int64_t)) + scan_workspace_size(n) + 256;
}

int dps_tiles_assemble(const uint32_t* gathered, int32_t world, int64_t n_mids, int64_t n_tiles,
                       int64_t tiles_per_rank, int64_t ent_cap, uint32_t* tile_off,
                       uint32_t* tile_ent, int64_t ent_words, uint32_t* tile_maxc,
                       int64_t* tile_gmin, int32_t* status, void* ws, size_t ws_bytes,
                       void* stream) {
  DPS_REQUIRE(world >= 1 && n_mids >= 0 && n_tiles >= 0 && tiles_per_rank >= 1 &&
                  tiles_per_rank * world >= n_tiles && ent_cap >= 0 && ent_words >= 0,
              DPS_ERR_INVALID, "bad assemble shape");
  DPS_REQUIRE(gathered && tile_off && tile_ent && status, DPS_ERR_INVALID, "null array");
  auto st = static_cast<hipStream_t>(stream);
  const int64_t cap = (ent_cap + 3) / 4 * 4;
  const int64_t words = SliceLayout(n_mids, tiles_per_rank, cap).words;
  const int64_t n = n_mids * world;
  Carve cv(ws, ws_bytes);
  int64_t* run = cv.take<int64_t>(static_cast<size_t>(n + 1));
  int64_t* base = cv.take<int64_t>(static_cast<size_t>(n + 1));
  const size_t sb = scan_workspace_size(n);
  void* sws = cv.take<char>(sb);
  DPS_REQUIRE(cv.ok, DPS_ERR_WORKSPACE, "workspace too small (%zu bytes)", ws_bytes);
  if (n > 0) {
    k_tiles_runs<<<grid_for(n, kBlock), kBlock, 0, st>>>(gathered, words, world, n_mids, n_tiles,
                                                         tiles_per_rank, cap, run, status);
    DPS_LAUNCHED();
  }
  DPS_HIP_RET(scan_exclusive<int64_t>(run, base, n, sws, sb, st));
  k_tiles_offsets<<<grid_for(n_mids * n_tiles + 1, kBlock), kBlock, 0, st>>>(
      gathered, words, world, n_mids, n_tiles, tiles_per_rank, cap, base, ent_words, status,
      tile_off, tile_maxc, tile_gmin);
  DPS_LAUNCHED();
  if (n > 0) {
    k_tiles_copy<<<grid_for(n * kWave, kBlock, 8192), kBlock, 0, st>>>(
        gathered, words, world, n_mids, n_tiles, tiles_per_rank, cap, base, ent_words, status,
        tile_ent);
    DPS_LAUNCHED();
  }
  return DPS_OK;
}

}  // extern "C"
