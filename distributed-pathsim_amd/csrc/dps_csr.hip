// Typed incidence extraction, typed CSR build (sort + unique = the motif's
// distinct), expand-sort-compress SpGEMM C = W_AP . W_PX, and the global-walk
// vectors s, g.  SURVEY.md §8a rows A2-A4.
#include "dps_common.hpp"

#include <cstdlib>

namespace dps {
namespace {

constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;
// ints staged in LDS by the long-segment path (56 KiB of dynamic LDS; it is
// reached through a generic pointer shared with the in-place global path, so it
// stays below 64 KiB: a 128 KiB static array faulted there, while ds_* access to
// 144 KiB static LDS is fine in k_col_sums_wide)
constexpr int kSegLdsCap = 14336;

__device__ __forceinline__ int64_t bound_from(const int64_t* dev, int64_t host) {
  return dev ? *dev : host;
}

// ---------------------------------------------------------------------------
// A2: typed incidence extraction (DPathSim_APVPA.py:78-84).  Wave-aggregated
// atomic append: one atomic per wave per output list.
#ifndef DPS_EXTRACT_PER
#define DPS_EXTRACT_PER 16
#endif
constexpr int kExtractPer = DPS_EXTRACT_PER;   // edges per lane per wave chunk (<= 32)

__global__ __launch_bounds__(kBlock) void k_extract(
    const int32_t* __restrict__ src, const int32_t* __restrict__ dst,
    const uint8_t* __restrict__ rel, int64_t n, const uint8_t* __restrict__ ntype,
    const int32_t* __restrict__ rowid, const int32_t* __restrict__ colid,
    int32_t* __restrict__ ap_r, int32_t* __restrict__ ap_c, unsigned long long* n_ap,
    int32_t* __restrict__ px_r, int32_t* __restrict__ px_c, unsigned long long* n_px) {
  // A wave owns chunks of kExtractPer*64 consecutive edges: pass 1 classifies
  // them (flags kept as bitmasks), one atomicAdd per output list reserves the
  // chunk's slots, pass 2 writes the pairs in edge order within the chunk.
  __shared__ unsigned long long cnt_s[2][kWavesPerBlock];
  __shared__ unsigned long long base_s[2];
  const int lane = lane_id();
  const int wave = threadIdx.x / kWave;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWavesPerBlock;
  constexpr int64_t kChunk = static_cast<int64_t>(kExtractPer) * kWave;
  // block-uniform trip count: every wave of a block reaches the barriers
  const int64_t blk0 = static_cast<int64_t>(blockIdx.x) * kWavesPerBlock * kChunk;
  for (int64_t cb = blk0; cb < n; cb += nwaves * kChunk) {
    const int64_t c0 = cb + wave * kChunk;
    uint32_t f_ap = 0, f_px = 0;
    int c_ap = 0, c_px = 0;
#pragma unroll
    for (int u = 0; u < kExtractPer; ++u) {
      const int64_t i = c0 + u * kWave + lane;
      bool is_ap = false, is_px = false;
      if (i < n) {
        const int32_t s = src[i], d = dst[i];
        const uint8_t r = rel[i];
        const uint8_t td = ntype[d];
        is_ap = (r == DPS_R_AP) && (td == DPS_T_PAPER);
        is_px = (r == DPS_R_PX) && (ntype[s] == DPS_T_PAPER) && (td == DPS_T_MID);
      }
      const uint64_t m_ap = ballot(is_ap), m_px = ballot(is_px);
      f_ap |= is_ap ? (1u << u) : 0u;
      f_px |= is_px ? (1u << u) : 0u;
      c_ap += __popcll(m_ap);
      c_px += __popcll(m_px);
    }
    // one reservation per block and list (the counters are hot addresses):
    // wave w's slots follow waves 0..w-1 of the same block iteration
    __syncthreads();   // the previous iteration's reads of cnt_s are done
    if (lane == 0) { cnt_s[0][wave] = c_ap; cnt_s[1][wave] = c_px; }
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long t_ap = 0, t_px = 0;
#pragma unroll
      for (int w = 0; w < kWavesPerBlock; ++w) { t_ap += cnt_s[0][w]; t_px += cnt_s[1][w]; }
      base_s[0] = t_ap ? atomicAdd(n_ap, t_ap) : 0ull;
      base_s[1] = t_px ? atomicAdd(n_px, t_px) : 0ull;
    }
    __syncthreads();
    int64_t o_ap = static_cast<int64_t>(base_s[0]), o_px = static_cast<int64_t>(base_s[1]);
#pragma unroll
    for (int w = 0; w < kWavesPerBlock; ++w)
      if (w < wave) { o_ap += cnt_s[0][w]; o_px += cnt_s[1][w]; }
#pragma unroll
    for (int u = 0; u < kExtractPer; ++u) {
      const int64_t i = c0 + u * kWave + lane;
      const bool is_ap = (f_ap >> u) & 1u, is_px = (f_px >> u) & 1u;
      const uint64_t m_ap = ballot(is_ap), m_px = ballot(is_px);
      if (is_ap) {
        const int64_t o = o_ap + mbcnt(m_ap);
        ap_r[o] = rowid[src[i]];
        ap_c[o] = colid[dst[i]];
      }
      if (is_px) {
        const int64_t o = o_px + mbcnt(m_px);
        px_r[o] = colid[src[i]];
        px_c[o] = colid[dst[i]];
      }
      o_ap += __popcll(m_ap);
      o_px += __popcll(m_px);
    }
  }
}

// ---------------------------------------------------------------------------
// Counting-sort scatter of (row, col) pairs into row segments.
__global__ __launch_bounds__(kBlock) void k_count_rows(const int32_t* __restrict__ rows,
                                                       int64_t cap, const int64_t* n_dev,
                                                       uint32_t* __restrict__ cnt) {
  const int64_t n = bound_from(n_dev, cap);
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * kBlock)
    atomicAdd(&cnt[rows[i]], 1u);
}

__global__ __launch_bounds__(kBlock) void k_scatter_rows(
    const int32_t* __restrict__ rows, const int32_t* __restrict__ cols, int64_t cap,
    const int64_t* n_dev, const int64_t* __restrict__ seg_ptr, uint32_t* __restrict__ cursor,
    int32_t* __restrict__ tmp) {
  const int64_t n = bound_from(n_dev, cap);
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * kBlock) {
    const int32_t r = rows[i];
    tmp[seg_ptr[r] + atomicAdd(&cursor[r], 1u)] = cols[i];
  }
}

// Two-level counting sort by row without global atomics (the per-pair global
// atomics of k_count_rows / k_scatter_rows run at the fabric's atomic rate,
// ~150-190 us per 7.5 M pairs on MI355X).  Level 1 buckets the pairs by row
// range (2^rb rows per bucket) with LDS histograms per block of kL1Chunk pairs,
// one exclusive scan over the [bucket][block] counts, and LDS cursors; level 2
// is one workgroup per bucket: an LDS histogram of its rows, a block scan that
// writes the bucket's seg_ptr entries directly (bucket start + local prefix),
// and an LDS-cursor scatter of the columns into their row segments.  The order
// inside a row segment is unspecified (seg_unique sorts it).
constexpr int kL1Chunk = 4096;        // pairs per level-1 block (kBlock threads x 16)
constexpr int kMaxBuckets = 4096;
constexpr int kMaxRbShift = 12;       // rows per bucket <= 4096 (level-2 LDS histogram)
// Pairs per level-1 bucket (at most; the bound is the raw edge count): 32768
// with a 1024-thread level-2 block -- config3's CSR 0.54 -> 0.44 ms against 8192
// with 256 threads (longer runs per bucket in the level-1 scatter, fewer
// level-1 counters to zero; rows-per-bucket sweep in
// profiles/r04/build4/csr_bucket_sweep.txt).
constexpr double kBucketPairs = 32768.0;
constexpr int kRowsBlock = 1024;

__global__ __launch_bounds__(kBlock) void k_bucket_hist(const int32_t* __restrict__ rows,
                                                        int64_t cap, const int64_t* n_dev,
                                                        int rb, int n_buckets, int64_t n_blocks,
                                                        uint32_t* __restrict__ H) {
  __shared__ uint32_t h[kMaxBuckets];
  for (int b = threadIdx.x; b < n_buckets; b += kBlock) h[b] = 0;
  __syncthreads();
  const int64_t n = bound_from(n_dev, cap);
  const int64_t i0 = static_cast<int64_t>(blockIdx.x) * kL1Chunk;
  const int64_t i1 = min(i0 + kL1Chunk, n);
  for (int64_t i = i0 + threadIdx.x; i < i1; i += kBlock) atomicAdd(&h[rows[i] >> rb], 1u);
  __syncthreads();
  for (int b = threadIdx.x; b < n_buckets; b += kBlock)
    H[static_cast<int64_t>(b) * n_blocks + blockIdx.x] = h[b];
}

// The block's pairs are first ordered by bucket in LDS (local counting sort),
// then written out run by run, so consecutive threads write consecutive
// addresses of a bucket's range instead of ~4 scattered pairs per bucket.
__global__ __launch_bounds__(kBlock) void k_bucket_scatter(
    const int32_t* __restrict__ rows, const int32_t* __restrict__ cols, int64_t cap,
    const int64_t* n_dev, int rb, int n_buckets, int64_t n_blocks,
    const int64_t* __restrict__ Hoff, int32_t* __restrict__ trow, int32_t* __restrict__ tcol) {
  __shared__ uint32_t cur[kMaxBuckets];     // local exclusive offsets, then cursors
  __shared__ uint32_t loc0[kMaxBuckets];    // local exclusive offsets (kept)
  __shared__ int32_t srow[kL1Chunk], scol[kL1Chunk];
  __shared__ uint32_t wsum[kWavesPerBlock];
  const int64_t n = bound_from(n_dev, cap);
  const int64_t i0 = static_cast<int64_t>(blockIdx.x) * kL1Chunk;
  const int64_t i1 = min(i0 + kL1Chunk, n);
  if (i0 >= i1) return;   // block-uniform
  const int m = static_cast<int>(i1 - i0);
  for (int b = threadIdx.x; b < n_buckets; b += kBlock) cur[b] = 0;
  __syncthreads();
  constexpr int kPer = kL1Chunk / kBlock;
  int32_t r[kPer], c[kPer];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int i = threadIdx.x + q * kBlock;
    r[q] = i < m ? rows[i0 + i] : -1;
    c[q] = i < m ? cols[i0 + i] : 0;
  }
#pragma unroll
  for (int q = 0; q < kPer; ++q)
    if (r[q] >= 0) atomicAdd(&cur[r[q] >> rb], 1u);
  __syncthreads();
  // exclusive scan of the local histogram (thread t: buckets [t*kq, (t+1)*kq))
  constexpr int kq = kMaxBuckets / kBlock;
  const int lane = lane_id(), wave = threadIdx.x / kWave;
  uint32_t h[kq], sum = 0;
#pragma unroll
  for (int q = 0; q < kq; ++q) {
    const int b = threadIdx.x * kq + q;
    h[q] = b < n_buckets ? cur[b] : 0u;
    sum += h[q];
  }
  const uint32_t inc = wave_inclusive_sum(sum);
  if (lane == kWave - 1) wsum[wave] = inc;
  __syncthreads();
  uint32_t run = inc - sum;
  for (int w = 0; w < wave; ++w) run += wsum[w];
#pragma unroll
  for (int q = 0; q < kq; ++q) {
    const int b = threadIdx.x * kq + q;
    if (b < n_buckets) { cur[b] = run; loc0[b] = run; }
    run += h[q];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    if (r[q] < 0) continue;
    const uint32_t pos = atomicAdd(&cur[r[q] >> rb], 1u);
    srow[pos] = r[q];
    scol[pos] = c[q];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < m; i += kBlock) {
    const int32_t rr = srow[i];
    const int b = rr >> rb;
    const int64_t o = Hoff[static_cast<int64_t>(b) * n_blocks + blockIdx.x] + (i - loc0[b]);
    trow[o] = rr;
    tcol[o] = scol[i];
  }
}

template <int BT>
__global__ __launch_bounds__(BT) void k_bucket_rows(
    const int32_t* __restrict__ trow, const int32_t* __restrict__ tcol, int rb, int64_t n_rows,
    int64_t n_blocks, const int64_t* __restrict__ Hoff, int64_t* __restrict__ seg_ptr,
    int32_t* __restrict__ seg) {
  constexpr int kBlock = BT, kWavesPerBlock = BT / kWave;
  __shared__ uint32_t cnt[1 << kMaxRbShift];
  __shared__ uint32_t wsum[kWavesPerBlock];
  const int64_t b = blockIdx.x;
  const int64_t r0 = b << rb;
  const int nr = static_cast<int>(min(static_cast<int64_t>(1) << rb, n_rows - r0));
  const int64_t s = Hoff[b * n_blocks], e = Hoff[(b + 1) * n_blocks];
  for (int r = threadIdx.x; r < nr; r += kBlock) cnt[r] = 0;
  __syncthreads();
  for (int64_t i = s + threadIdx.x; i < e; i += kBlock)
    atomicAdd(&cnt[trow[i] - r0], 1u);
  __syncthreads();
  // exclusive scan of cnt[0..nr): thread t owns the run [t*per, (t+1)*per)
  constexpr int kPer = (1 << kMaxRbShift) / kBlock;
  const int lane = lane_id(), wave = threadIdx.x / kWave;
  const int q0 = threadIdx.x * kPer;
  uint32_t loc[kPer], sum = 0;
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    loc[q] = q0 + q < nr ? cnt[q0 + q] : 0u;
    sum += loc[q];
  }
  const uint32_t inc = wave_inclusive_sum(sum);
  if (lane == kWave - 1) wsum[wave] = inc;
  __syncthreads();
  uint32_t run = inc - sum;
  for (int w = 0; w < wave; ++w) run += wsum[w];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    if (q0 + q < nr) {
      cnt[q0 + q] = run;
      seg_ptr[r0 + q0 + q] = s + run;
    }
    run += loc[q];
  }
  if (r0 + nr == n_rows && threadIdx.x == 0) seg_ptr[n_rows] = e;
  __syncthreads();
  for (int64_t i = s + threadIdx.x; i < e; i += kBlock) {
    const uint32_t pos = atomicAdd(&cnt[trow[i] - r0], 1u);
    seg[s + pos] = tcol[i];
  }
}

// Level-1 geometry for n_rows rows and at most cap pairs: about 8192 pairs per
// bucket, at most kMaxBuckets buckets (ok = false: use the atomic path).
struct BucketPlan {
  bool ok;
  int rb;
  int n_buckets;
  int64_t n_blocks;
};
BucketPlan bucket_plan(int64_t cap, int64_t n_rows) {
  BucketPlan P{false, 0, 0, 0};
  if (cap <= 0 || n_rows <= 0) return P;
  int rb = 0;
  while (rb < kMaxRbShift && (static_cast<double>(cap) * (1ll << (rb + 1))) / n_rows <= kBucketPairs) ++rb;
  while (rb < kMaxRbShift && ((n_rows + (1ll << rb) - 1) >> rb) > kMaxBuckets) ++rb;
  const int64_t nbk = (n_rows + (1ll << rb) - 1) >> rb;
  if (nbk > kMaxBuckets) return P;
  P.ok = true;
  P.rb = rb;
  P.n_buckets = static_cast<int>(nbk);
  P.n_blocks = (cap + kL1Chunk - 1) / kL1Chunk;
  return P;
}

// Column sums (and author-entry counts) for more mids than one LDS range:
// block (x, y) reduces the mids [y*kWideMids, (y+1)*kWideMids) of entry chunk
// x in 144 KiB of LDS (u64 sums, u32 counts; one 1024-thread block per CU),
// then flushes one global atomic per nonzero (block, mid).  The chunks are
// few (about two blocks per CU over all ranges), so the flush stays small;
// every range re-reads c_col (config4: 17 ranges x 118 MB).  Replaces a
// per-4096-entry LDS hash whose flush was one scattered global atomic per
// entry (config4: 2.29 ms).
constexpr int kWideBlock = 1024;
constexpr int kWideMids = 12288;

__global__ __launch_bounds__(kWideBlock) void k_col_sums_wide(const int64_t* __restrict__ c_ptr,
                                                              const int32_t* __restrict__ c_col,
                                                              const int32_t* __restrict__ c_val,
                                                              int64_t n_rows, int64_t n_mids,
                                                              unsigned long long* __restrict__ s,
                                                              int64_t n_count_rows,
                                                              unsigned* __restrict__ n_v) {
  __shared__ unsigned long long h[kWideMids];
  __shared__ unsigned hc[kWideMids];
  const int64_t m0 = static_cast<int64_t>(blockIdx.y) * kWideMids;
  const int m = static_cast<int>(min(static_cast<int64_t>(kWideMids), n_mids - m0));
  for (int i = threadIdx.x; i < m; i += kWideBlock) { h[i] = 0; hc[i] = 0; }
  __syncthreads();
  const int64_t b0 = c_ptr[0], nnz = c_ptr[n_rows] - b0;
  const int64_t ncnt = n_v ? c_ptr[n_count_rows] - b0 : 0;
  // the block's entries [J0, J1) in absolute positions, read as int4 groups
  // (groups straddling a chunk edge are read by both blocks, each taking its
  // own entries); c_val only for the entries in range
  const int64_t per = ((nnz + gridDim.x - 1) / gridDim.x + 3) & ~int64_t(3);
  const int64_t J0 = b0 + min(static_cast<int64_t>(blockIdx.x) * per, nnz);
  const int64_t J1 = b0 + min(static_cast<int64_t>(blockIdx.x + 1) * per, nnz);
  const int64_t Jc = b0 + ncnt;
  const int64_t Jend = b0 + nnz;
  const bool vec = (reinterpret_cast<uintptr_t>(c_col) & 15) == 0;
  for (int64_t q = (J0 >> 2) + threadIdx.x; (q << 2) < J1; q += kWideBlock) {
    int32_t col4[4];
    if (vec && (q << 2) + 4 <= Jend) {          // never past the last entry
      const int4 cv = reinterpret_cast<const int4*>(c_col)[q];
      col4[0] = cv.x; col4[1] = cv.y; col4[2] = cv.z; col4[3] = cv.w;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t j = (q << 2) + e;
        col4[e] = (j >= J0 && j < J1) ? c_col[j] : -1;
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t j = (q << 2) + e;
      const uint32_t d = static_cast<uint32_t>(col4[e] - m0);
      if (j >= J0 && j < J1 && d < static_cast<uint32_t>(m)) {
        atomicAdd(&h[d], static_cast<unsigned long long>(c_val[j]));
        if (j < Jc) atomicAdd(&hc[d], 1u);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < m; i += kWideBlock) {
    if (h[i]) atomicAdd(&s[m0 + i], h[i]);
    if (n_v && hc[i]) atomicAdd(&n_v[m0 + i], hc[i]);
  }
}

// Column sums for many mids without re-reading C per mid range (round 5):
// the entries are first bucketed by mid range (kWideMids mids each) -- a
// per-block LDS count of each range's entries, one exclusive scan of the
// [range][block] counts, and a scatter of packed (local mid | author flag,
// C) pairs with LDS cursors -- then every range is reduced from its own
// bucket in LDS as in k_col_sums_wide.  Three reads and one write of 8 B per
// entry instead of one 4 B read per entry per range (config4: 17 ranges).
constexpr int kCsBlocks = 1024;       // blocks of the count / scatter passes
constexpr int kCsMaxRanges = 4096;    // n_mids <= kCsMaxRanges * kWideMids
constexpr uint32_t kCsAuthor = 0x80000000u;

__device__ __forceinline__ void cs_chunk(int64_t nnz, int64_t& j0, int64_t& j1) {
  const int64_t per = (nnz + gridDim.x - 1) / gridDim.x;
  j0 = min(static_cast<int64_t>(blockIdx.x) * per, nnz);
  j1 = min(j0 + per, nnz);
}

__global__ __launch_bounds__(kBlock) void k_cs_count(const int64_t* __restrict__ c_ptr,
                                                     const int32_t* __restrict__ c_col,
                                                     int64_t n_rows, int n_ranges,
                                                     uint32_t* __restrict__ cnt) {
  __shared__ uint32_t h[kCsMaxRanges];
  for (int r = threadIdx.x; r < n_ranges; r += kBlock) h[r] = 0;
  __syncthreads();
  const int64_t b0 = c_ptr[0];
  int64_t j0, j1;
  cs_chunk(c_ptr[n_rows] - b0, j0, j1);
  for (int64_t j = j0 + threadIdx.x; j < j1; j += kBlock)
    atomicAdd(&h[c_col[b0 + j] / kWideMids], 1u);
  __syncthreads();
  for (int r = threadIdx.x; r < n_ranges; r += kBlock) cnt[static_cast<int64_t>(r) * gridDim.x + blockIdx.x] = h[r];
}

__global__ __launch_bounds__(kBlock) void k_cs_scatter(const int64_t* __restrict__ c_ptr,
                                                       const int32_t* __restrict__ c_col,
                                                       const int32_t* __restrict__ c_val,
                                                       int64_t n_rows, int64_t n_count_rows,
                                                       int n_ranges, const int64_t* __restrict__ off,
                                                       int64_t cap, uint2* __restrict__ pairs) {
  __shared__ unsigned long long cur[kCsMaxRanges];
  for (int r = threadIdx.x; r < n_ranges; r += kBlock)
    cur[r] = static_cast<unsigned long long>(off[static_cast<int64_t>(r) * gridDim.x + blockIdx.x]);
  __syncthreads();
  const int64_t b0 = c_ptr[0];
  const int64_t ncnt = c_ptr[n_count_rows] - b0;
  int64_t j0, j1;
  cs_chunk(c_ptr[n_rows] - b0, j0, j1);
  for (int64_t j = j0 + threadIdx.x; j < j1; j += kBlock) {
    const int32_t v = c_col[b0 + j];
    const int r = v / kWideMids;
    const unsigned long long pos = atomicAdd(&cur[r], 1ull);
    if (pos < static_cast<unsigned long long>(cap))
      pairs[pos] = make_uint2(static_cast<uint32_t>(v - r * kWideMids) | (j < ncnt ? kCsAuthor : 0u),
                            static_cast<uint32_t>(c_val[b0 + j]));
  }
}

// block (x, y): its share of range y's bucket [off[y * nb], off[(y + 1) * nb]).
__global__ __launch_bounds__(kWideBlock) void k_cs_range(const uint2* __restrict__ pairs,
                                                         const int64_t* __restrict__ off, int nb,
                                                         const int64_t* __restrict__ c_ptr,
                                                         int64_t n_rows, int64_t cap, int64_t n_mids,
                                                         unsigned long long* __restrict__ s,
                                                         unsigned* __restrict__ n_v) {
  __shared__ unsigned long long h[kWideMids];
  __shared__ unsigned hc[kWideMids];
  const int64_t m0 = static_cast<int64_t>(blockIdx.y) * kWideMids;
  const int m = static_cast<int>(min(static_cast<int64_t>(kWideMids), n_mids - m0));
  for (int i = threadIdx.x; i < m; i += kWideBlock) { h[i] = 0; hc[i] = 0; }
  __syncthreads();
  const int64_t total = c_ptr[n_rows] - c_ptr[0];
  const int64_t a = min(off[static_cast<int64_t>(blockIdx.y) * nb], cap);
  const int64_t b = min(blockIdx.y + 1 < gridDim.y ? off[static_cast<int64_t>(blockIdx.y + 1) * nb] : total, cap);
  const int64_t per = (b - a + gridDim.x - 1) / gridDim.x;
  const int64_t q0 = a + min(static_cast<int64_t>(blockIdx.x) * per, b - a);
  const int64_t q1 = min(q0 + per, b);
  for (int64_t q = q0 + threadIdx.x; q < q1; q += kWideBlock) {
    const uint2 e = pairs[q];
    const uint32_t d = e.x & ~kCsAuthor;
    atomicAdd(&h[d], static_cast<unsigned long long>(e.y));
    if (n_v && (e.x & kCsAuthor)) atomicAdd(&hc[d], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < m; i += kWideBlock) {
    if (h[i]) atomicAdd(&s[m0 + i], h[i]);
    if (n_v && hc[i]) atomicAdd(&n_v[m0 + i], hc[i]);
  }
}

__host__ __forceinline__ dim3 col_sums_wide_grid(int64_t n_mids) {
  const unsigned ny = static_cast<unsigned>((n_mids + kWideMids - 1) / kWideMids);
  const unsigned nx = ny >= 512 ? 1u : 512u / ny;
  return dim3(nx, ny);
}

// ---------------------------------------------------------------------------
// Segmented sort + unique (+ run lengths).
// Tiny segments (2..16): one lane each, a 16-input bitonic network in registers.
constexpr int kLaneSeg = 16;
// medium segments (65 .. 256): one wave each, LDS bitonic.  Longer ones go to
// the 1024-thread rank sort: a wave's bitonic over 1024 entries (55 dependent
// LDS steps of 8 pairs per lane) took ~50 us alone and set k_seg_mid's time.
constexpr int kMidSeg = 256;

template <int N>
__device__ __forceinline__ void lane_sort_unique(int32_t* __restrict__ data,
                                                 int32_t* __restrict__ counts, int64_t beg,
                                                 int len, int64_t* __restrict__ uniq_out,
                                                 const SegSrc& src) {
  int32_t v[N];
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = i < len ? seg_in(data, src, beg + i) : INT_MAX;
#pragma unroll
  for (int k = 2; k <= N; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const int l = i ^ j;
        if (l > i) {
          const int32_t a = v[i], b = v[l];
          const bool up = (i & k) == 0;
          v[i] = up ? min(a, b) : max(a, b);
          v[l] = up ? max(a, b) : min(a, b);
        }
      }
    }
  }
  int u = 0;
  int run = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    if (i < len) {
      const bool first = i == 0 || v[i] != v[i - 1];
      if (first) {
        if (i > 0 && counts) counts[beg + u - 1] = run;
        data[beg + u] = v[i];
        ++u;
        run = 1;
      } else {
        ++run;
      }
    }
  }
  if (counts) counts[beg + u - 1] = run;
  *uniq_out = u;
}

// Short segments (<= 64): one wave, bitonic sort in registers.
__global__ __launch_bounds__(kBlock) void k_seg_short(int32_t* __restrict__ data,
                                                      int32_t* __restrict__ counts,
                                                      const int64_t* __restrict__ seg_ptr,
                                                      int64_t n_seg, int64_t* __restrict__ uniq,
                                                      int32_t* __restrict__ long_list,
                                                      unsigned* __restrict__ n_long,
                                                      int32_t* __restrict__ mid_list,
                                                      unsigned* __restrict__ n_mid,
                                                      SegSrc src) {
  // Triage 64 segments per wave, one per lane (coalesced seg_ptr reads): empty
  // and single-element segments are finished by their lane, medium ones (65 ..
  // kMidSeg, when mid_list is given) go to the wave-level kernel, long ones to
  // the block-level kernel, and the rest are sorted one at a time by the
  // whole wave.  Most segments of the typed CSR builds are empty (non-author
  // rows) or single (one venue per paper).
  const int lane = lane_id();
  const int64_t wave0 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWavesPerBlock;
  for (int64_t s0 = wave0 * kWave; s0 < n_seg; s0 += nwaves * kWave) {
    const int64_t sl = s0 + lane;
    int64_t bl = 0;
    int ll = 0;
    if (sl < n_seg) {
      bl = seg_ptr[sl];
      ll = static_cast<int>(seg_ptr[sl + 1] - bl);
      if (ll <= 1) {
        uniq[sl] = ll;
        if (ll == 1) {
          if (counts) counts[bl] = 1;
          if (src.map) data[bl] = seg_in(data, src, bl);
        }
      } else if (ll <= kLaneSeg) {
        lane_sort_unique<kLaneSeg>(data, counts, bl, ll, uniq + sl, src);
      } else if (ll <= 2 * kLaneSeg) {
        // 17 .. 32 (config4's expansions: 30 on average): a 32-input network
        // per lane -- 64 segments at once instead of one per wave
        lane_sort_unique<2 * kLaneSeg>(data, counts, bl, ll, uniq + sl, src);
      } else if (mid_list && ll > kWave && ll <= kMidSeg) {
        mid_list[atomicAdd(n_mid, 1u)] = static_cast<int32_t>(sl);
      } else if (ll > kWave) {
        long_list[atomicAdd(n_long, 1u)] = static_cast<int32_t>(sl);
      }
    }
    uint64_t todo = ballot(ll > 2 * kLaneSeg && ll <= kWave);
    while (todo) {
      const int sl_lane = __ffsll(static_cast<long long>(todo)) - 1;
      todo &= todo - 1;
      const int64_t s = s0 + sl_lane;
      const int64_t beg = readlane(bl, sl_lane);
      const int len = readlane(ll, sl_lane);
      int v = lane < len ? seg_in(data, src, beg + lane) : INT_MAX;
      v = wave_bitonic_sort(v);
      const int prev = __shfl_up(v, 1, kWave);
      const bool first = lane < len && (lane == 0 || v != prev);
      const uint64_t mask = ballot(first);
      if (first) {
        const int rank = mbcnt(mask);
        data[beg + rank] = v;
        if (counts) {
          const uint64_t above = mask & ~((2ull << lane) - 1ull);
          const int next = above ? (__ffsll(static_cast<long long>(above)) - 1) : len;
          counts[beg + rank] = next - lane;
        }
      }
      if (lane == 0) uniq[s] = __popcll(mask);
    }
  }
}

// Medium segments (65 .. kMidSeg): one wave each, staged in 1 KiB of LDS,
// bitonic network with virtual +inf padding (as block_bitonic_sort, at wave
// scope), then unique (+ run lengths) in 64-entry strips.  A 1024-thread
// block per segment (k_seg_long) left 90 % of its threads idle on config4's
// 54 k segments of about 114 entries.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(kBlock) void k_seg_mid(int32_t* __restrict__ data,
                                                    int32_t* __restrict__ counts,
                                                    const int64_t* __restrict__ seg_ptr,
                                                    int64_t* __restrict__ uniq,
                                                    const int32_t* __restrict__ mid_list,
                                                    const unsigned* __restrict__ n_mid,
                                                    SegSrc src) {
  __shared__ int32_t buf[kWavesPerBlock][kMidSeg];
  const int lane = lane_id();
  const int wave = threadIdx.x / kWave;
  int32_t* a = buf[wave];
  const unsigned nm = *n_mid;
  const unsigned nwaves = gridDim.x * kWavesPerBlock;
  for (unsigned li = blockIdx.x * kWavesPerBlock + wave; li < nm; li += nwaves) {
    const int64_t sg = mid_list[li];
    const int64_t beg = seg_ptr[sg];
    const int len = static_cast<int>(seg_ptr[sg + 1] - beg);
    for (int i = lane; i < len; i += kWave) a[i] = seg_in(data, src, beg + i);
    wave_lds_sync();
    int n2 = kWave;
    while (n2 < len) n2 <<= 1;
    const int half_n = n2 >> 1;
    for (int k = 2; k <= n2; k <<= 1) {
      const int half = k >> 1;
      for (int p = lane; p < half_n; p += kWave) {
        const int blk = p / half, off = p - blk * half;
        const int i = blk * k + off, j = blk * k + k - 1 - off;
        if (j < len) {
          const int32_t ai = a[i], aj = a[j];
          if (aj < ai) { a[i] = aj; a[j] = ai; }
        }
      }
      wave_lds_sync();
      for (int jd = half >> 1; jd > 0; jd >>= 1) {
        for (int p = lane; p < half_n; p += kWave) {
          const int blk = p / jd, off = p - blk * jd;
          const int i = blk * 2 * jd + off, j = i + jd;
          if (j < len) {
            const int32_t ai = a[i], aj = a[j];
            if (aj < ai) { a[i] = aj; a[j] = ai; }
          }
        }
        wave_lds_sync();
      }
    }
    int carry = 0;
    for (int c0 = 0; c0 < len; c0 += kWave) {
      const int i = c0 + lane;
      const bool valid = i < len;
      const int32_t v = valid ? a[i] : 0;
      const bool first = valid && (i == 0 || v != a[i - 1]);
      const uint64_t mask = ballot(first);
      if (first) {
        const int r = carry + mbcnt(mask);
        data[beg + r] = v;
        if (counts) {
          // run length: next head in this strip, else the strip's first head
          // of the next one is found below through the position array
          const uint64_t above = mask & ~((2ull << lane) - 1ull);
          int next;
          if (above) {
            next = c0 + __ffsll(static_cast<long long>(above)) - 1;
          } else {
            next = len;
            for (int q = c0 + kWave; q < len; ++q)
              if (a[q] != a[q - 1]) { next = q; break; }
          }
          counts[beg + r] = next - i;
        }
      }
      carry += __popcll(mask);
    }
    if (lane == 0) uniq[sg] = carry;
    wave_lds_sync();
  }
}

// Ascending bitonic network over a[0..len) with virtual +inf padding to a
// power of two.  Every comparator puts the minimum at the lower index
// ("flip" formulation), so padded slots never need to be materialised.
__device__ void block_bitonic_sort(int32_t* a, int len) {
  int n2 = 1;
  while (n2 < len) n2 <<= 1;
  const int half_n = n2 >> 1;
  for (int k = 2; k <= n2; k <<= 1) {
    const int half = k >> 1;
    for (int p = threadIdx.x; p < half_n; p += blockDim.x) {
      const int blk = p / half, off = p - blk * half;
      const int i = blk * k + off, j = blk * k + k - 1 - off;
      if (j < len) {
        const int32_t ai = a[i], aj = a[j];
        if (aj < ai) { a[i] = aj; a[j] = ai; }
      }
    }
    __syncthreads();
    for (int jd = half >> 1; jd > 0; jd >>= 1) {
      for (int p = threadIdx.x; p < half_n; p += blockDim.x) {
        const int blk = p / jd, off = p - blk * jd;
        const int i = blk * 2 * jd + off, j = i + jd;
        if (j < len) {
          const int32_t ai = a[i], aj = a[j];
          if (aj < ai) { a[i] = aj; a[j] = ai; }
        }
      }
      __syncthreads();
    }
  }
}

// Block-wide exclusive scan of one int per thread (NW waves per block).
template <int NW>
__device__ int64_t block_excl_scan_int(int v, int64_t* lds_w, int64_t* total) {
  const int lane = lane_id();
  const int wave = threadIdx.x / kWave;
  int64_t inc = wave_inclusive_sum(static_cast<int64_t>(v));
  if (lane == kWave - 1) lds_w[wave] = inc;
  __syncthreads();
  int64_t off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const int64_t x = lds_w[w];
    off += w < wave ? x : 0;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return off + inc - v;
}

// Long segments: one 1024-thread block each; staged in LDS when they fit, else
// sorted in place in global memory.  Then unique (+ run lengths) in
// block-sized chunks.
constexpr int kLongBlock = 1024;
constexpr int kRankSortMax = kLongBlock;   // segments up to this long: rank sort

__global__ __launch_bounds__(kLongBlock) void k_seg_long(int32_t* __restrict__ data,
                                                         int32_t* __restrict__ counts,
                                                         const int64_t* __restrict__ seg_ptr,
                                                         int64_t* __restrict__ uniq,
                                                         const int32_t* __restrict__ long_list,
                                                         const unsigned* __restrict__ n_long,
                                                         unsigned* __restrict__ next,
                                                         SegSrc src) {
  extern __shared__ __attribute__((aligned(16))) int32_t lds_seg[];
  constexpr int kNW = kLongBlock / kWave;
  __shared__ int64_t lds_w[kNW];
  __shared__ int32_t lds_prev;
  __shared__ unsigned li_s;
  const unsigned nl = *n_long;
  // segments are taken from a queue (one atomic per segment): a block that
  // drew a few long ones does not hold up the rest of the list
  for (;;) {
    if (threadIdx.x == 0) li_s = atomicAdd(next, 1u);
    __syncthreads();
    const unsigned li = li_s;
    __syncthreads();
    if (li >= nl) break;
    const int64_t s = long_list[li];
    const int64_t beg = seg_ptr[s];
    const int len = static_cast<int>(seg_ptr[s + 1] - beg);
    int32_t* a;
    if (len <= kRankSortMax) {
      // rank sort (no barrier per phase): element i goes to the number of
      // elements before it in (value, index) order; 4 values per LDS read
      const int i = threadIdx.x;
      const int32_t x = i < len ? seg_in(data, src, beg + i) : INT_MAX;
      const int len4 = (len + 3) & ~3;
      lds_seg[i] = x;                              // padding: INT_MAX at index >= len
      __syncthreads();
      int r = 0;
      for (int j = 0; j < len4; j += 4) {
        const int4 v = *reinterpret_cast<const int4*>(lds_seg + j);
        r += (v.x < x || (v.x == x && j < i)) ? 1 : 0;
        r += (v.y < x || (v.y == x && j + 1 < i)) ? 1 : 0;
        r += (v.z < x || (v.z == x && j + 2 < i)) ? 1 : 0;
        r += (v.w < x || (v.w == x && j + 3 < i)) ? 1 : 0;
      }
      if (i < len) lds_seg[kRankSortMax + r] = x;  // padding ranks are never below len
      __syncthreads();
      a = lds_seg + kRankSortMax;
    } else if (len <= kSegLdsCap) {
      for (int i = threadIdx.x; i < len; i += kLongBlock) lds_seg[i] = seg_in(data, src, beg + i);
      __syncthreads();
      a = lds_seg;
      block_bitonic_sort(a, len);
    } else {
      a = data + beg;
      if (src.map) {                      // gather the segment into place first
        for (int i = threadIdx.x; i < len; i += kLongBlock) a[i] = seg_in(data, src, beg + i);
        __syncthreads();
      }
      block_bitonic_sort(a, len);
    }
    int64_t carry = 0;
    for (int c0 = 0; c0 < len; c0 += kLongBlock) {
      const int i = c0 + threadIdx.x;
      const bool valid = i < len;
      const int32_t v = valid ? a[i] : 0;
      int32_t prev = 0;
      if (valid && i > 0) prev = (threadIdx.x == 0) ? lds_prev : a[i - 1];
      const bool first = valid && (i == 0 || v != prev);
      __syncthreads();  // every read of this chunk happens before any write below
      if (threadIdx.x == kLongBlock - 1 || i == len - 1) lds_prev = v;
      int64_t tot;
      const int64_t rank = carry + block_excl_scan_int<kNW>(first ? 1 : 0, lds_w, &tot);
      if (first) {
        data[beg + rank] = v;
        if (counts) counts[beg + rank] = i;  // position for now; turned into lengths below
      }
      carry += tot;
      __syncthreads();
    }
    if (counts) {
      for (int64_t u0 = 0; u0 < carry; u0 += kLongBlock) {
        const int64_t u = u0 + threadIdx.x;
        int32_t here = 0, next = 0;
        if (u < carry) {
          here = counts[beg + u];
          next = (u + 1 < carry) ? counts[beg + u + 1] : len;
        }
        __syncthreads();
        if (u < carry) counts[beg + u] = next - here;
        __syncthreads();
      }
    }
    if (threadIdx.x == 0) uniq[s] = carry;
    __syncthreads();
  }
}

// Long segments over a small key range (values < key_range <= kHistKeys, or
// INT_MAX = "none", which sorts last): an LDS histogram per segment replaces
// the sort -- the nonzero bins in order ARE the sorted distinct values and
// their run lengths (the single-mid SpGEMM's venue rows).
constexpr int kHistKeys = 8192;

__global__ __launch_bounds__(kBlock) void k_seg_long_hist(int32_t* __restrict__ data,
                                                          int32_t* __restrict__ counts,
                                                          const int64_t* __restrict__ seg_ptr,
                                                          int64_t* __restrict__ uniq,
                                                          const int32_t* __restrict__ long_list,
                                                          const unsigned* __restrict__ n_long,
                                                          int key_range, SegSrc src) {
  __shared__ uint32_t hist[kHistKeys + 1];
  __shared__ int64_t lds_w[kWavesPerBlock];
  const int nb = key_range + 1;                      // bin key_range: INT_MAX
  const int per = (nb + kBlock - 1) / kBlock;        // bins per thread (contiguous)
  const unsigned nl = *n_long;
  // static assignment (a per-segment queue measured 2x slower here: the
  // segments are short and uniform, the queue's two barriers are not)
  for (unsigned li = blockIdx.x; li < nl; li += gridDim.x) {
    const int64_t s = long_list[li];
    const int64_t beg = seg_ptr[s];
    const int len = static_cast<int>(seg_ptr[s + 1] - beg);
    for (int b = threadIdx.x; b < nb; b += kBlock) hist[b] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < len; i += kBlock) {
      const int32_t v = seg_in(data, src, beg + i);
      atomicAdd(&hist[v < key_range ? v : key_range], 1u);
    }
    __syncthreads();
    const int b0 = threadIdx.x * per;
    int nz = 0;
    for (int q = 0; q < per; ++q) nz += (b0 + q < nb && hist[b0 + q] != 0) ? 1 : 0;
    int64_t tot;
    int64_t rank = block_excl_scan_int<kWavesPerBlock>(nz, lds_w, &tot);
    for (int q = 0; q < per; ++q) {
      const int b = b0 + q;
      if (b >= nb) break;
      const uint32_t h = hist[b];
      if (!h) continue;
      data[beg + rank] = b < key_range ? b : INT_MAX;
      if (counts) counts[beg + rank] = static_cast<int32_t>(h);
      ++rank;
    }
    if (threadIdx.x == 0) uniq[s] = tot;
    __syncthreads();
  }
}

// Compact segment heads into the final CSR arrays.
__global__ __launch_bounds__(kBlock) void k_compact(const int32_t* __restrict__ tmp,
                                                    const int32_t* __restrict__ tmp_cnt,
                                                    const int64_t* __restrict__ seg_ptr,
                                                    const int64_t* __restrict__ out_ptr,
                                                    int64_t n_seg, int32_t* __restrict__ col,
                                                    int32_t* __restrict__ val) {
  const int64_t wave0 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWavesPerBlock;
  for (int64_t s0 = wave0 * kWave; s0 < n_seg; s0 += nwaves * kWave)
    compact_heads_wave(tmp, tmp_cnt, seg_ptr, out_ptr, n_seg, col, val, s0);
}

__global__ void k_copy_scalar(const int64_t* src, int64_t* dst) { *dst = *src; }

// ---------------------------------------------------------------------------
// SpGEMM (expand-sort-compress).  Wave per output row.
__device__ __forceinline__ int64_t out_row_src(const int32_t* rows, int64_t i) {
  return rows ? static_cast<int64_t>(rows[i]) : i;
}

// Both expansion kernels: a wave owns 64 consecutive output rows and walks
// the concatenation of their AP segments in 64-entry strips (a lane finds its
// row by a binary search over the segment offsets, wave_owner), one paper per
// lane.  A lane per row with the wave taking rows of more than 32 papers left
// each lane a serial chain of dependent loads per paper (config4: 582 us for
// the expansion, 160 us for its lengths).
struct ApStrips {
  int64_t b;        // this lane's row: first AP entry, ...
  uint32_t excl;    // ... its offset in the wave's concatenation
  uint32_t total;   // the wave's AP entries
};
__device__ __forceinline__ ApStrips ap_strips(const int64_t* __restrict__ ap_ptr,
                                              const int32_t* __restrict__ rows, int64_t x,
                                              int64_t n_out) {
  ApStrips a{0, 0, 0};
  uint32_t len = 0;
  if (x < n_out) {
    const int64_t r = out_row_src(rows, x);
    a.b = ap_ptr[r];
    len = static_cast<uint32_t>(ap_ptr[r + 1] - a.b);
  }
  const uint32_t incl = wave_inclusive_sum(len);
  a.excl = incl - len;
  a.total = readlane(incl, kWave - 1);
  return a;
}

__global__ __launch_bounds__(kBlock) void k_expand_len(const int64_t* __restrict__ ap_ptr,
                                                       const int32_t* __restrict__ ap_col,
                                                       const int32_t* __restrict__ rows,
                                                       int64_t n_out,
                                                       const int64_t* __restrict__ px_ptr,
                                                       int64_t* __restrict__ e_len,
                                                       unsigned long long* e_total) {
  // per-row sums in LDS by owner lane; one atomic per block for the total
  __shared__ unsigned long long acc[kWavesPerBlock][kWave];
  const int lane = lane_id();
  const int wave = threadIdx.x / kWave;
  const int64_t wave0 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWavesPerBlock;
  int64_t lane_total = 0;
  for (int64_t i0 = wave0 * kWave; i0 < n_out; i0 += nwaves * kWave) {
    const int64_t x = i0 + lane;
    const ApStrips a = ap_strips(ap_ptr, rows, x, n_out);
    acc[wave][lane] = 0;
    __builtin_amdgcn_wave_barrier();
    for (uint32_t e0 = 0; e0 < a.total; e0 += kWave) {
      const uint32_t i = e0 + static_cast<uint32_t>(lane);
      const int o = wave_owner(a.excl, i);   // every lane takes part in the shuffles
      const int64_t bo = readlane_var(a.b, o);
      const uint32_t eo = static_cast<uint32_t>(__shfl(static_cast<int>(a.excl), o, kWave));
      if (i < a.total) {
        const int32_t p = ap_col[bo + (i - eo)];
        const int64_t c = px_ptr[p + 1] - px_ptr[p];
        if (c) atomicAdd(&acc[wave][o], static_cast<unsigned long long>(c));
        lane_total += c;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (x < n_out && e_len) e_len[x] = static_cast<int64_t>(acc[wave][lane]);
    __builtin_amdgcn_wave_barrier();
  }
  __shared__ int64_t part[kWavesPerBlock];
  const int64_t wave_total = wave_sum(lane_total);
  if (lane == 0) part[wave] = wave_total;
  __syncthreads();
  if (threadIdx.x == 0 && e_total) {
    int64_t t = 0;
#pragma unroll
    for (int w = 0; w < kWavesPerBlock; ++w) t += part[w];
    if (t) atomicAdd(e_total, static_cast<unsigned long long>(t));
  }
}

__global__ __launch_bounds__(kBlock) void k_expand(const int64_t* __restrict__ ap_ptr,
                                                   const int32_t* __restrict__ ap_col,
                                                   const int32_t* __restrict__ rows, int64_t n_out,
                                                   const int64_t* __restrict__ px_ptr,
                                                   const int32_t* __restrict__ px_col,
                                                   const int64_t* __restrict__ exp_ptr,
                                                   int32_t* __restrict__ tmp) {
  // the expansion of rows i0 .. i0+63 is contiguous from exp_ptr[i0], in the
  // order of the concatenated AP entries: a running carry + a wave scan of the
  // papers' mid counts place each paper's mids
  const int lane = lane_id();
  const int64_t wave0 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWavesPerBlock;
  for (int64_t i0 = wave0 * kWave; i0 < n_out; i0 += nwaves * kWave) {
    const ApStrips a = ap_strips(ap_ptr, rows, i0 + lane, n_out);
    int64_t carry = exp_ptr[i0];
    for (uint32_t e0 = 0; e0 < a.total; e0 += kWave) {
      const uint32_t i = e0 + static_cast<uint32_t>(lane);
      const int o = wave_owner(a.excl, i);
      const int64_t bo = readlane_var(a.b, o);
      const uint32_t eo = static_cast<uint32_t>(__shfl(static_cast<int>(a.excl), o, kWave));
      int64_t pb = 0;
      uint32_t pl = 0;
      if (i < a.total) {
        const int32_t p = ap_col[bo + (i - eo)];
        pb = px_ptr[p];
        pl = static_cast<uint32_t>(px_ptr[p + 1] - pb);
      }
      // the strip's mids, 64 at a time: each lane copies one (its paper by a
      // second owner search), so the loads of a strip are all in flight at
      // once instead of one paper's mids one after another per lane
      const uint32_t inc = wave_inclusive_sum(pl);
      const uint32_t pex = inc - pl;
      const uint32_t tot = readlane(inc, kWave - 1);
      for (uint32_t m0 = 0; m0 < tot; m0 += kWave) {
        const uint32_t m = m0 + static_cast<uint32_t>(lane);
        const int po = wave_owner(pex, m);
        const int64_t pbo = readlane_var(pb, po);
        const uint32_t peo = static_cast<uint32_t>(__shfl(static_cast<int>(pex), po, kWave));
        if (m < tot) tmp[carry + m] = px_col[pbo + (m - peo)];
      }
      carry += tot;
    }
  }
}

// ---------------------------------------------------------------------------
// A4: s[v] = sum_{(p,v) in PX} indeg_AP(p);  g = C.s, diag, stats.
__global__ __launch_bounds__(kBlock) void k_paper_indeg(const int64_t* __restrict__ ap_ptr,
                                                        const int32_t* __restrict__ ap_col,
                                                        int64_t n_rows,
                                                        int32_t* __restrict__ indeg) {
  const int64_t nnz = ap_ptr[n_rows];
  for (int64_t j = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; j < nnz;
       j += static_cast<int64_t>(gridDim.x) * kBlock)
    atomicAdd(&indeg[ap_col[j]], 1);
}

constexpr int64_t kMidLds = 6144;   // mids whose walk sums are reduced in LDS per block

__global__ __launch_bounds__(kBlock) void k_mid_walks(const int64_t* __restrict__ px_ptr,
                                                      const int32_t* __restrict__ px_col,
                                                      int64_t n_papers, int64_t n_mids,
                                                      const int32_t* __restrict__ indeg,
                                                      unsigned long long* __restrict__ s) {
  // per-block partial sums in LDS (hot venues would otherwise take one global
  // atomic per paper), flushed with one atomic per mid and block
  __shared__ unsigned long long s_lds[kMidLds];
  const bool lds = n_mids <= kMidLds;
  if (lds)
    for (int64_t i = threadIdx.x; i < n_mids; i += kBlock) s_lds[i] = 0;
  __syncthreads();
  for (int64_t p = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; p < n_papers;
       p += static_cast<int64_t>(gridDim.x) * kBlock) {
    const int d = indeg[p];
    if (d == 0) continue;
    for (int64_t j = px_ptr[p]; j < px_ptr[p + 1]; ++j) {
      if (lds) atomicAdd(&s_lds[px_col[j]], static_cast<unsigned long long>(d));
      else atomicAdd(&s[px_col[j]], static_cast<unsigned long long>(d));
    }
  }
  __syncthreads();
  if (lds)
    for (int64_t i = threadIdx.x; i < n_mids; i += kBlock)
      if (s_lds[i]) atomicAdd(&s[i], s_lds[i]);
}

__global__ __launch_bounds__(kBlock) void k_global_walks(const int64_t* __restrict__ c_ptr,
                                                         const int32_t* __restrict__ c_col,
                                                         const int32_t* __restrict__ c_val,
                                                         int64_t n_rows,
                                                         const int64_t* __restrict__ s,
                                                         int64_t* __restrict__ g,
                                                         int64_t* __restrict__ diag,
                                                         unsigned long long* __restrict__ stats,
                                                         const unsigned* __restrict__ n_v,
                                                         int64_t* __restrict__ terms) {
  // A wave owns 64 consecutive rows, whose entries are one contiguous range of
  // C: it walks that range in coalesced 64-entry strips (a lane finds its row
  // by a 6-step search over the row offsets) and sums per row in LDS, so a
  // heavy row costs strips, not one lane's serial loop.  (Measured slower: an
  // LDS start-marker + DPP max-scan instead of the search, +6 %; a wave
  // reduction for strips inside one row instead of its LDS atomics, +13 %.)
  __shared__ unsigned long long acc_g[kWavesPerBlock][kWave];
  __shared__ unsigned long long acc_d[kWavesPerBlock][kWave];
  __shared__ unsigned long long acc_t[kWavesPerBlock][kWave];   // row work (n_v given)
  const int lane = lane_id();
  const int wave = threadIdx.x / kWave;
  int64_t max_c = 0, max_d = 0, max_g = 0;
  const int64_t wave0 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWavesPerBlock;
  for (int64_t r0 = wave0 * kWave; r0 < n_rows; r0 += nwaves * kWave) {
    const int64_t x = r0 + lane;
    const int64_t base = c_ptr[r0];
    const int64_t xe = x < n_rows ? x : n_rows;
    const uint32_t excl = static_cast<uint32_t>(c_ptr[xe] - base);
    const uint32_t total = static_cast<uint32_t>(
        c_ptr[r0 + kWave < n_rows ? r0 + kWave : n_rows] - base);
    acc_g[wave][lane] = 0;
    acc_d[wave][lane] = 0;
    acc_t[wave][lane] = 0;
    __builtin_amdgcn_wave_barrier();
    for (uint32_t e0 = 0; e0 < total; e0 += kWave) {
      const uint32_t i = e0 + lane;
      const int o = wave_owner(excl, i);   // every lane takes part in the shuffles
      if (i < total) {
        const int64_t j = base + i;
        const int64_t c = c_val[j];
        const int32_t v = c_col[j];
        atomicAdd(&acc_g[wave][o], static_cast<unsigned long long>(c * s[v]));
        atomicAdd(&acc_d[wave][o], static_cast<unsigned long long>(c * c));
        if (n_v) atomicAdd(&acc_t[wave][o], static_cast<unsigned long long>(n_v[v]));
        max_c = c > max_c ? c : max_c;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (x < n_rows) {
      const int64_t gx = static_cast<int64_t>(acc_g[wave][lane]);
      const int64_t dx = static_cast<int64_t>(acc_d[wave][lane]);
      g[x] = gx;
      if (diag) diag[x] = dx;
      if (terms) terms[x] = static_cast<int64_t>(acc_t[wave][lane]);
      max_d = dx > max_d ? dx : max_d;
      max_g = gx > max_g ? gx : max_g;
    }
    __builtin_amdgcn_wave_barrier();
  }
  max_c = wave_max(max_c);
  max_d = wave_max(max_d);
  max_g = wave_max(max_g);
  if (lane == 0 && stats) {
    atomic_max_filtered(&stats[DPS_STAT_MAX_C], static_cast<unsigned long long>(max_c));
    atomic_max_filtered(&stats[DPS_STAT_MAX_DIAG], static_cast<unsigned long long>(max_d));
    atomic_max_filtered(&stats[DPS_STAT_MAX_G], static_cast<unsigned long long>(max_g));
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && stats)
    stats[DPS_STAT_NNZ_C] = static_cast<unsigned long long>(c_ptr[n_rows] - c_ptr[0]);
}

// Per-row work estimate of the hot kernel: terms[x] = sum_{v in x} n_v, n_v =
// nnz of column v of C (over rows [0, n_rows)).  Column counts are reduced in
// LDS per block (one global atomic per mid and block) when they fit.
constexpr int64_t kColLds = 8192;

__global__ __launch_bounds__(kBlock) void k_col_counts(const int64_t* __restrict__ c_ptr,
                                                       const int32_t* __restrict__ c_col,
                                                       int64_t n_rows, int64_t n_mids,
                                                       unsigned* __restrict__ n_v) {
  // block (x, y) counts the mids [y*kColLds, (y+1)*kColLds) of its share of the
  // entries in LDS: hot (heavy) mids never take one global atomic per entry
  __shared__ unsigned h[kColLds];
  const int64_t m0 = static_cast<int64_t>(blockIdx.y) * kColLds;
  const int64_t m1 = min(m0 + kColLds, n_mids);
  for (int64_t i = threadIdx.x; i < m1 - m0; i += kBlock) h[i] = 0;
  __syncthreads();
  const int64_t nnz = c_ptr[n_rows] - c_ptr[0];
  for (int64_t j = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; j < nnz;
       j += static_cast<int64_t>(gridDim.x) * kBlock) {
    const int64_t v = c_col[c_ptr[0] + j];
    if (v >= m0 && v < m1) atomicAdd(&h[v - m0], 1u);
  }
  __syncthreads();
  for (int64_t i = threadIdx.x; i < m1 - m0; i += kBlock)
    if (h[i]) atomicAdd(&n_v[m0 + i], h[i]);
}

__global__ __launch_bounds__(kBlock) void k_row_terms(const int64_t* __restrict__ c_ptr,
                                                      const int32_t* __restrict__ c_col,
                                                      int64_t n_rows,
                                                      const unsigned* __restrict__ n_v,
                                                      int64_t* __restrict__ terms) {
  // as k_global_walks: a wave owns 64 consecutive rows and walks their entries
  // in coalesced 64-entry strips, summing per row in LDS
  __shared__ unsigned long long acc[kWavesPerBlock][kWave];
  const int lane = lane_id();
  const int wave = threadIdx.x / kWave;
  const int64_t wave0 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWavesPerBlock;
  for (int64_t r0 = wave0 * kWave; r0 < n_rows; r0 += nwaves * kWave) {
    const int64_t x = r0 + lane;
    const int64_t base = c_ptr[r0];
    const int64_t xe = x < n_rows ? x : n_rows;
    const uint32_t excl = static_cast<uint32_t>(c_ptr[xe] - base);
    const uint32_t total = static_cast<uint32_t>(
        c_ptr[r0 + kWave < n_rows ? r0 + kWave : n_rows] - base);
    acc[wave][lane] = 0;
    __builtin_amdgcn_wave_barrier();
    for (uint32_t e0 = 0; e0 < total; e0 += kWave) {
      const uint32_t i = e0 + lane;
      const int o = wave_owner(excl, i);   // every lane takes part in the shuffles
      if (i < total) atomicAdd(&acc[wave][o], static_cast<unsigned long long>(n_v[c_col[base + i]]));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (x < n_rows) terms[x] = static_cast<int64_t>(acc[wave][lane]);
    __builtin_amdgcn_wave_barrier();
  }
}

// s[v] = sum over rows [0, n_rows) of C[r,v] (column sums of C over every AP
// row = the mid walks of the global-walk motif): per-block LDS sums, one
// global atomic per mid and block when the mids fit in LDS.
constexpr int64_t kSumLds = 6144;

__global__ __launch_bounds__(kBlock) void k_col_sums(const int64_t* __restrict__ c_ptr,
                                                     const int32_t* __restrict__ c_col,
                                                     const int32_t* __restrict__ c_val,
                                                     int64_t n_rows, int64_t n_mids,
                                                     unsigned long long* __restrict__ s,
                                                     int64_t n_count_rows,
                                                     unsigned* __restrict__ n_v) {
  // block (x, y) sums the mids [y*kSumLds, (y+1)*kSumLds) of its share of the
  // entries in LDS, one global atomic per mid and block; with n_v it also
  // counts the entries of rows [0, n_count_rows) per mid (the hot kernel's
  // row-work weights: C^T holds the author rows only)
  __shared__ unsigned long long h[kSumLds];
  __shared__ unsigned hc[kSumLds];
  const int64_t m0 = static_cast<int64_t>(blockIdx.y) * kSumLds;
  const int64_t m1 = min(m0 + kSumLds, n_mids);
  for (int64_t i = threadIdx.x; i < m1 - m0; i += kBlock) { h[i] = 0; hc[i] = 0; }
  __syncthreads();
  const int64_t b0 = c_ptr[0], nnz = c_ptr[n_rows] - b0;
  const int64_t ncnt = n_v ? c_ptr[n_count_rows] - b0 : 0;
  for (int64_t j = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; j < nnz;
       j += static_cast<int64_t>(gridDim.x) * kBlock) {
    const int64_t v = c_col[b0 + j];
    if (v >= m0 && v < m1) {
      atomicAdd(&h[v - m0], static_cast<unsigned long long>(c_val[b0 + j]));
      if (j < ncnt) atomicAdd(&hc[v - m0], 1u);
    }
  }
  __syncthreads();
  for (int64_t i = threadIdx.x; i < m1 - m0; i += kBlock) {
    if (h[i]) atomicAdd(&s[m0 + i], h[i]);
    if (n_v && hc[i]) atomicAdd(&n_v[m0 + i], hc[i]);
  }
}

}  // namespace

// ---------------------------------------------------------------------------
size_t seg_unique_workspace_size(int64_t n_seg) {
  return 2 * align_up(static_cast<size_t>(n_seg > 0 ? n_seg : 1) * sizeof(int32_t)) + 512;
}

hipError_t seg_unique(int32_t* data, int32_t* counts, const int64_t* seg_ptr, int64_t n_seg,
                      int64_t* uniq, void* ws, size_t ws_bytes, hipStream_t stream,
                      int key_range, SegSrc src) {
  Carve c(ws, ws_bytes);
  int32_t* long_list = c.take<int32_t>(n_seg > 0 ? n_seg : 1);
  int32_t* mid_list = c.take<int32_t>(n_seg > 0 ? n_seg : 1);
  unsigned* n_long = c.take<unsigned>(4);   // [0] long list length, [1] queue head, [2] medium
  if (!c.ok) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(n_long, 0, 4 * sizeof(unsigned), stream);
  if (e != hipSuccess) return e;
  if (n_seg <= 0) return hipSuccess;
  // small key range: every segment over 64 goes to the LDS-histogram kernel
  const bool hist = key_range > 0 && key_range <= kHistKeys;
  k_seg_short<<<grid_for(n_seg, kBlock), kBlock, 0, stream>>>(
      data, counts, seg_ptr, n_seg, uniq, long_list, n_long, hist ? nullptr : mid_list, n_long + 2,
      src);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (!hist) {
    k_seg_mid<<<2048, kBlock, 0, stream>>>(data, counts, seg_ptr, uniq, mid_list, n_long + 2,
                                           src);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if (hist) {
    k_seg_long_hist<<<1024, kBlock, 0, stream>>>(data, counts, seg_ptr, uniq, long_list, n_long,
                                                 key_range, src);
    return hipGetLastError();
  }
  k_seg_long<<<512, kLongBlock, kSegLdsCap * sizeof(int32_t), stream>>>(
      data, counts, seg_ptr, uniq, long_list, n_long, n_long + 1, src);
  return hipGetLastError();
}

}  // namespace dps

using namespace dps;

extern "C" {

int dps_extract_incidence(const int32_t* edge_src, const int32_t* edge_dst,
                          const uint8_t* edge_rel, int64_t n_edges, const uint8_t* node_type,
                          const int32_t* node_rowid, const int32_t* node_colid, int64_t n_nodes,
                          int32_t* ap_row, int32_t* ap_col, int64_t* n_ap, int32_t* px_row,
                          int32_t* px_col, int64_t* n_px, void* stream) {
  DPS_REQUIRE(n_edges >= 0 && n_nodes >= 0, DPS_ERR_INVALID, "negative size");
  DPS_REQUIRE(n_ap && n_px, DPS_ERR_INVALID, "null count output");
  auto st = static_cast<hipStream_t>(stream);
  {
    FillSet fs;   // both counters in one launch
    fs.add(n_ap, 2, 0u);
    fs.add(n_px, 2, 0u);
    DPS_HIP_RET(fill_set(fs, st));
  }
  if (n_edges == 0) return DPS_OK;
  DPS_REQUIRE(edge_src && edge_dst && edge_rel && node_type && node_rowid && node_colid &&
                  ap_row && ap_col && px_row && px_col,
              DPS_ERR_INVALID, "null array");
  k_extract<<<grid_for((n_edges + kExtractPer - 1) / kExtractPer, kBlock), kBlock, 0, st>>>(
      edge_src, edge_dst, edge_rel, n_edges, node_type, node_rowid, node_colid, ap_row, ap_col,
      reinterpret_cast<unsigned long long*>(n_ap), px_row, px_col,
      reinterpret_cast<unsigned long long*>(n_px));
  DPS_LAUNCHED();
  return DPS_OK;
}

size_t dps_csr_build_workspace_size(int64_t n_pairs, int64_t n_rows) {
  const size_t nr = static_cast<size_t>(n_rows > 0 ? n_rows : 1);
  const size_t np = static_cast<size_t>(n_pairs > 0 ? n_pairs : 1);
  size_t s = 0;
  const BucketPlan B = bucket_plan(n_pairs, n_rows);
  if (B.ok) {
    const size_t nh = static_cast<size_t>(B.n_buckets) * static_cast<size_t>(B.n_blocks);
    s += align_up((nh + 1) * sizeof(uint32_t));   // H
    s += align_up((nh + 1) * sizeof(int64_t));    // Hoff
    s += align_up(scan_workspace_size(static_cast<int64_t>(nh)));
    s += 2 * align_up(np * sizeof(int32_t));      // bucketed rows, cols
  }
  s += align_up(nr * sizeof(uint32_t));           // cnt
  s += align_up(nr * sizeof(uint32_t));           // cursor
  s += align_up((nr + 1) * sizeof(int64_t));      // seg_ptr
  s += align_up(nr * sizeof(int64_t));            // uniq
  s += align_up(np * sizeof(int32_t));            // tmp
  s += align_up(scan_workspace_size(n_rows + 1));
  s += align_up(seg_unique_workspace_size(n_rows));
  return s + 1024;
}

int dps_csr_build(const int32_t* rows, const int32_t* cols, int64_t n_pairs,
                  const int64_t* n_pairs_dev, int64_t n_rows, int64_t* row_ptr, int32_t* col_out,
                  int64_t* nnz_out, void* ws, size_t ws_bytes, void* stream) {
  DPS_REQUIRE(n_pairs >= 0 && n_rows >= 0, DPS_ERR_INVALID, "negative size");
  DPS_REQUIRE(n_rows < INT32_MAX, DPS_ERR_OVERFLOW, "n_rows %lld exceeds int32",
              static_cast<long long>(n_rows));
  DPS_REQUIRE(row_ptr && nnz_out, DPS_ERR_INVALID, "null output");
  DPS_REQUIRE(reinterpret_cast<uintptr_t>(ws) % 256 == 0, DPS_ERR_WORKSPACE,
              "workspace not 256-byte aligned");
  DPS_REQUIRE(ws_bytes >= dps_csr_build_workspace_size(n_pairs, n_rows), DPS_ERR_WORKSPACE,
              "csr_build workspace too small: %zu < %zu", ws_bytes,
              dps_csr_build_workspace_size(n_pairs, n_rows));
  auto st = static_cast<hipStream_t>(stream);
  Carve c(ws, ws_bytes);
  const int64_t nr = n_rows > 0 ? n_rows : 1;
  uint32_t* cnt = c.take<uint32_t>(nr);
  uint32_t* cursor = c.take<uint32_t>(nr);
  int64_t* seg_ptr = c.take<int64_t>(nr + 1);
  int64_t* uniq = c.take<int64_t>(nr);
  int32_t* tmp = c.take<int32_t>(n_pairs > 0 ? n_pairs : 1);
  const size_t scan_ws = scan_workspace_size(n_rows + 1);
  void* sws = c.take<char>(scan_ws);
  const size_t seg_ws = seg_unique_workspace_size(n_rows);
  void* gws = c.take<char>(seg_ws);
  DPS_REQUIRE(c.ok, DPS_ERR_WORKSPACE, "csr_build workspace carve failed");

  const BucketPlan B = bucket_plan(n_pairs, n_rows);
  bool atomic_path = false;   // A/B (profiling build only): the per-pair atomic path
#ifdef DPS_PROFILE
  if (const char* env = std::getenv("DPATHSIM_CSR_ATOMIC")) atomic_path = std::atoi(env) != 0;
#endif
  if (B.ok && !atomic_path) {
    DPS_REQUIRE(rows && cols, DPS_ERR_INVALID, "null input pairs");
    const int64_t nh = static_cast<int64_t>(B.n_buckets) * B.n_blocks;
    uint32_t* H = c.take<uint32_t>(nh + 1);
    int64_t* Hoff = c.take<int64_t>(nh + 1);
    const size_t hs_ws = scan_workspace_size(nh);
    void* hws = c.take<char>(hs_ws);
    int32_t* trow = c.take<int32_t>(n_pairs);
    int32_t* tcol = c.take<int32_t>(n_pairs);
    DPS_REQUIRE(c.ok, DPS_ERR_WORKSPACE, "csr_build workspace carve failed");
    k_bucket_hist<<<static_cast<unsigned>(B.n_blocks), kBlock, 0, st>>>(
        rows, n_pairs, n_pairs_dev, B.rb, B.n_buckets, B.n_blocks, H);
    DPS_LAUNCHED();
    DPS_HIP_RET(scan_exclusive<uint32_t>(H, Hoff, nh, hws, hs_ws, st));
    k_bucket_scatter<<<static_cast<unsigned>(B.n_blocks), kBlock, 0, st>>>(
        rows, cols, n_pairs, n_pairs_dev, B.rb, B.n_buckets, B.n_blocks, Hoff, trow, tcol);
    DPS_LAUNCHED();
    k_bucket_rows<kRowsBlock><<<static_cast<unsigned>(B.n_buckets), kRowsBlock, 0, st>>>(
        trow, tcol, B.rb, n_rows, B.n_blocks, Hoff, seg_ptr, tmp);
    DPS_LAUNCHED();
  } else {
    DPS_HIP_RET(hipMemsetAsync(cnt, 0, nr * sizeof(uint32_t), st));
    DPS_HIP_RET(hipMemsetAsync(cursor, 0, nr * sizeof(uint32_t), st));
    if (n_pairs > 0) {
      DPS_REQUIRE(rows && cols, DPS_ERR_INVALID, "null input pairs");
      k_count_rows<<<grid_for(n_pairs, kBlock), kBlock, 0, st>>>(rows, n_pairs, n_pairs_dev, cnt);
      DPS_LAUNCHED();
    }
    DPS_HIP_RET(scan_exclusive<uint32_t>(cnt, seg_ptr, n_rows, sws, scan_ws, st));
    if (n_pairs > 0) {
      k_scatter_rows<<<grid_for(n_pairs, kBlock), kBlock, 0, st>>>(rows, cols, n_pairs, n_pairs_dev,
                                                                   seg_ptr, cursor, tmp);
      DPS_LAUNCHED();
    }
  }
  DPS_HIP_RET(seg_unique(tmp, nullptr, seg_ptr, n_rows, uniq, gws, seg_ws, st));
  DPS_HIP_RET(scan_exclusive<int64_t>(uniq, row_ptr, n_rows, sws, scan_ws, st));
  if (n_rows > 0) {
    k_compact<<<grid_for(n_rows, kBlock), kBlock, 0, st>>>(tmp, nullptr, seg_ptr, row_ptr,
                                                                   n_rows, col_out, nullptr);
    DPS_LAUNCHED();
  }
  k_copy_scalar<<<1, 1, 0, st>>>(row_ptr + n_rows, nnz_out);
  DPS_LAUNCHED();
  return DPS_OK;
}

int dps_spgemm_expand_size(const int64_t* ap_ptr, const int32_t* ap_col, const int32_t* rows,
                           int64_t n_out_rows, const int64_t* px_ptr, int64_t* e_total,
                           void* stream) {
  DPS_REQUIRE(n_out_rows >= 0, DPS_ERR_INVALID, "negative size");
  DPS_REQUIRE(e_total, DPS_ERR_INVALID, "null output");
  auto st = static_cast<hipStream_t>(stream);
  DPS_HIP_RET(hipMemsetAsync(e_total, 0, sizeof(int64_t), st));
  if (n_out_rows == 0) return DPS_OK;
  k_expand_len<<<grid_for(n_out_rows, kBlock, 1024), kBlock, 0, st>>>(   // <= 1024 hot atomics
      ap_ptr, ap_col, rows, n_out_rows, px_ptr, nullptr,
      reinterpret_cast<unsigned long long*>(e_total));
  DPS_LAUNCHED();
  return DPS_OK;
}

size_t dps_spgemm_workspace_size(int64_t n_out_rows, int64_t expand_cap) {
  const size_t n = static_cast<size_t>(n_out_rows > 0 ? n_out_rows : 1);
  const size_t e = static_cast<size_t>(expand_cap > 0 ? expand_cap : 1);
  size_t s = 0;
  s += align_up(n * sizeof(int64_t));         // e_len
  s += align_up((n + 1) * sizeof(int64_t));   // exp_ptr
  s += align_up(n * sizeof(int64_t));         // uniq
  s += align_up(e * sizeof(int32_t));         // tmp
  s += align_up(e * sizeof(int32_t));         // counts
  s += align_up(scan_workspace_size(n_out_rows + 1));
  s += align_up(seg_unique_workspace_size(n_out_rows));
  return s + 1024;
}

int dps_spgemm_count(const int64_t* ap_ptr, const int32_t* ap_col, const int32_t* rows,
                     int64_t n_out_rows, const int64_t* px_ptr, const int32_t* px_col,
                     int64_t n_papers, int64_t* c_ptr, int32_t* c_col, int32_t* c_val,
                     int64_t* c_nnz, int64_t expand_cap, void* ws, size_t ws_bytes,
                     void* stream) {
  (void)n_papers;
  DPS_REQUIRE(n_out_rows >= 0 && expand_cap >= 0, DPS_ERR_INVALID, "negative size");
  DPS_REQUIRE(c_ptr && c_nnz, DPS_ERR_INVALID, "null output");
  DPS_REQUIRE(reinterpret_cast<uintptr_t>(ws) % 256 == 0, DPS_ERR_WORKSPACE,
              "workspace not 256-byte aligned");
  DPS_REQUIRE(ws_bytes >= dps_spgemm_workspace_size(n_out_rows, expand_cap), DPS_ERR_WORKSPACE,
              "spgemm workspace too small");
  DPS_REQUIRE(!c_col == !c_val, DPS_ERR_INVALID, "c_col and c_val must both be set (numeric)");
  auto st = static_cast<hipStream_t>(stream);
  Carve c(ws, ws_bytes);
  const int64_t n = n_out_rows > 0 ? n_out_rows : 1;
  int64_t* e_len = c.take<int64_t>(n);
  int64_t* exp_ptr = c.take<int64_t>(n + 1);
  int64_t* uniq = c.take<int64_t>(n);
  int32_t* tmp = c.take<int32_t>(expand_cap > 0 ? expand_cap : 1);
  int32_t* cnt = c.take<int32_t>(expand_cap > 0 ? expand_cap : 1);
  const size_t scan_ws = scan_workspace_size(n_out_rows + 1);
  void* sws = c.take<char>(scan_ws);
  const size_t seg_ws = seg_unique_workspace_size(n_out_rows);
  void* gws = c.take<char>(seg_ws);
  DPS_REQUIRE(c.ok, DPS_ERR_WORKSPACE, "spgemm workspace carve failed");

  if (c_col == nullptr) {  // symbolic: expand, sort, unique+count; keep results in ws
    if (n_out_rows > 0) {
      k_expand_len<<<grid_for(n_out_rows, kBlock), kBlock, 0, st>>>(
          ap_ptr, ap_col, rows, n_out_rows, px_ptr, e_len, nullptr);
      DPS_LAUNCHED();
    }
    DPS_HIP_RET(scan_exclusive<int64_t>(e_len, exp_ptr, n_out_rows, sws, scan_ws, st));
    if (n_out_rows > 0) {
      k_expand<<<grid_for(n_out_rows, kBlock), kBlock, 0, st>>>(
          ap_ptr, ap_col, rows, n_out_rows, px_ptr, px_col, exp_ptr, tmp);
      DPS_LAUNCHED();
    }
    DPS_HIP_RET(seg_unique(tmp, cnt, exp_ptr, n_out_rows, uniq, gws, seg_ws, st));
    DPS_HIP_RET(scan_exclusive<int64_t>(uniq, c_ptr, n_out_rows, sws, scan_ws, st));
    k_copy_scalar<<<1, 1, 0, st>>>(c_ptr + n_out_rows, c_nnz);
    DPS_LAUNCHED();
    return DPS_OK;
  }
  if (n_out_rows > 0) {  // numeric: compact (workspace of the symbolic call, unmodified)
    k_compact<<<grid_for(n_out_rows, kBlock), kBlock, 0, st>>>(tmp, cnt, exp_ptr, c_ptr,
                                                                       n_out_rows, c_col, c_val);
    DPS_LAUNCHED();
  }
  return DPS_OK;
}

int dps_mid_walks(const int64_t* ap_ptr, const int32_t* ap_col, int64_t n_ap_rows,
                  const int64_t* px_ptr, const int32_t* px_col, int64_t n_papers, int64_t n_mids,
                  int32_t* paper_indeg_ws, int64_t* s, void* stream) {
  DPS_REQUIRE(n_ap_rows >= 0 && n_papers >= 0 && n_mids >= 0, DPS_ERR_INVALID, "negative size");
  auto st = static_cast<hipStream_t>(stream);
  if (n_mids > 0) DPS_HIP_RET(hipMemsetAsync(s, 0, n_mids * sizeof(int64_t), st));
  if (n_papers == 0) return DPS_OK;
  DPS_HIP_RET(hipMemsetAsync(paper_indeg_ws, 0, n_papers * sizeof(int32_t), st));
  k_paper_indeg<<<2048, kBlock, 0, st>>>(ap_ptr, ap_col, n_ap_rows, paper_indeg_ws);
  DPS_LAUNCHED();
  k_mid_walks<<<grid_for(n_papers, kBlock, 1024), kBlock, 0, st>>>(
      px_ptr, px_col, n_papers, n_mids, paper_indeg_ws, reinterpret_cast<unsigned long long*>(s));
  DPS_LAUNCHED();
  return DPS_OK;
}

int dps_global_walks(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                     int64_t n_rows, const int64_t* s, int64_t* g, int64_t* diag, int64_t* stats,
                     void* stream) {
  DPS_REQUIRE(n_rows >= 0, DPS_ERR_INVALID, "negative size");
  auto st = static_cast<hipStream_t>(stream);
  if (stats) DPS_HIP_RET(hipMemsetAsync(stats, 0, DPS_STATS_LEN * sizeof(int64_t), st));
  k_global_walks<<<grid_for(n_rows, kBlock), kBlock, 0, st>>>(
      c_ptr, c_col, c_val, n_rows, s, g, diag, reinterpret_cast<unsigned long long*>(stats),
      nullptr, nullptr);
  DPS_LAUNCHED();
  return DPS_OK;
}

// The bucketed column sums (more than kSumLds mids, at most kCsMaxRanges
// ranges of kWideMids) hold one 8-byte (mid | author flag, C) pair per C entry:
// 8 B x nnz_cap of HBM on top of the per-range counts; other shapes need none.
size_t dps_walks_workspace_size(int64_t nnz_cap, int64_t n_mids) {
  if (n_mids <= kSumLds || nnz_cap <= 0 ||
      n_mids > static_cast<int64_t>(kCsMaxRanges) * kWideMids)
    return 256;
  const int64_t nr = (n_mids + kWideMids - 1) / kWideMids;
  const int64_t m = nr * kCsBlocks;
  return align_up(static_cast<size_t>(m) * sizeof(uint32_t)) +
         align_up(static_cast<size_t>(m) * sizeof(int64_t)) + scan_workspace_size(m) +
         align_up(static_cast<size_t>(nnz_cap) * sizeof(uint2)) + 256;
}

int dps_walks_fused(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                    int64_t n_rows, int64_t n_authors, int64_t n_mids, int64_t* s,
                    uint32_t* n_v, int64_t* g, int64_t* diag, int64_t* terms, int64_t* stats,
                    void* stream) {
  return dps_walks_fused_ws(c_ptr, c_col, c_val, n_rows, n_authors, n_mids, s, n_v, g, diag,
                            terms, stats, 0, nullptr, 0, stream);
}

int dps_walks_fused_ws(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                       int64_t n_rows, int64_t n_authors, int64_t n_mids, int64_t* s,
                       uint32_t* n_v, int64_t* g, int64_t* diag, int64_t* terms, int64_t* stats,
                       int64_t nnz_cap, void* ws, size_t ws_bytes, void* stream) {
  DPS_REQUIRE(n_rows >= 0 && n_authors >= 0 && n_authors <= n_rows && n_mids >= 0,
              DPS_ERR_INVALID, "bad sizes");
  DPS_REQUIRE(c_ptr && g && (n_mids == 0 || (s && n_v)), DPS_ERR_INVALID, "null array");
  // more mids than the bucketed column sums cover (kCsMaxRanges ranges) take
  // the range-by-range k_col_sums_wide below, as without a workspace
  const bool bucketed = n_mids <= static_cast<int64_t>(kCsMaxRanges) * kWideMids;
  auto st = static_cast<hipStream_t>(stream);
  {
    FillSet fs;   // stats, s and n_v zeroed in one launch
    if (stats) fs.add(stats, 2 * DPS_STATS_LEN, 0u);
    if (n_mids > 0) {
      fs.add(s, 2 * n_mids, 0u);
      fs.add(n_v, n_mids, 0u);
    }
    DPS_HIP_RET(fill_set(fs, st));
  }
  if (n_mids > 0) {
    if (n_rows > 0 && n_mids > kSumLds && bucketed && ws != nullptr && nnz_cap > 0) {
      // bucketed by mid range (nnz_cap >= nnz C: the caller's bound, as for
      // the SpGEMM output; the scatter never writes past it)
      DPS_REQUIRE(ws_bytes >= dps_walks_workspace_size(nnz_cap, n_mids), DPS_ERR_WORKSPACE,
                  "walks workspace too small");
      DPS_REQUIRE(reinterpret_cast<uintptr_t>(ws) % 256 == 0, DPS_ERR_WORKSPACE,
                  "workspace not 256-byte aligned");
      const int nr = static_cast<int>((n_mids + kWideMids - 1) / kWideMids);
      const int64_t m = static_cast<int64_t>(nr) * kCsBlocks;
      Carve c(ws, ws_bytes);
      uint32_t* cnt = c.take<uint32_t>(m);
      int64_t* off = c.take<int64_t>(m);
      const size_t sws_bytes = scan_workspace_size(m);
      void* sws = c.take<char>(sws_bytes);
      uint2* pairs = c.take<uint2>(nnz_cap);
      DPS_REQUIRE(c.ok, DPS_ERR_WORKSPACE, "walks workspace carve failed");
      k_cs_count<<<kCsBlocks, kBlock, 0, st>>>(c_ptr, c_col, n_rows, nr, cnt);
      DPS_LAUNCHED();
      DPS_HIP_RET(scan_exclusive<uint32_t>(cnt, off, m, sws, sws_bytes, st));
      k_cs_scatter<<<kCsBlocks, kBlock, 0, st>>>(c_ptr, c_col, c_val, n_rows, n_authors, nr, off,
                                                 nnz_cap, pairs);
      DPS_LAUNCHED();
      const unsigned nx = nr >= 512 ? 1u : 512u / static_cast<unsigned>(nr);
      k_cs_range<<<dim3(nx, static_cast<unsigned>(nr)), kWideBlock, 0, st>>>(
          pairs, off, kCsBlocks, c_ptr, n_rows, nnz_cap, n_mids,
          reinterpret_cast<unsigned long long*>(s), n_v);
      DPS_LAUNCHED();
    } else if (n_rows > 0 && n_mids > kSumLds) {
      k_col_sums_wide<<<col_sums_wide_grid(n_mids), kWideBlock, 0, st>>>(
          c_ptr, c_col, c_val, n_rows, n_mids, reinterpret_cast<unsigned long long*>(s), n_authors,
          n_v);
      DPS_LAUNCHED();
    } else if (n_rows > 0) {
      k_col_sums<<<512, kBlock, 0, st>>>(c_ptr, c_col, c_val, n_rows, n_mids,
                                         reinterpret_cast<unsigned long long*>(s), n_authors, n_v);
      DPS_LAUNCHED();
    }
  }
  if (n_authors == 0) return DPS_OK;
  k_global_walks<<<grid_for(n_authors, kBlock), kBlock, 0, st>>>(
      c_ptr, c_col, c_val, n_authors, s, g, diag, reinterpret_cast<unsigned long long*>(stats),
      n_mids > 0 ? n_v : nullptr, terms);
  DPS_LAUNCHED();
  return DPS_OK;
}

int dps_col_sums(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                 int64_t n_rows, int64_t n_mids, int64_t* s, void* stream) {
  DPS_REQUIRE(n_rows >= 0 && n_mids >= 0, DPS_ERR_INVALID, "negative size");
  DPS_REQUIRE(c_ptr && (n_mids == 0 || s), DPS_ERR_INVALID, "null array");
  auto st = static_cast<hipStream_t>(stream);
  if (n_mids == 0) return DPS_OK;
  DPS_HIP_RET(hipMemsetAsync(s, 0, n_mids * sizeof(int64_t), st));
  if (n_rows == 0) return DPS_OK;
  if (n_mids > kSumLds) {
    k_col_sums_wide<<<col_sums_wide_grid(n_mids), kWideBlock, 0, st>>>(
        c_ptr, c_col, c_val, n_rows, n_mids, reinterpret_cast<unsigned long long*>(s), 0, nullptr);
  } else {
    k_col_sums<<<512, kBlock, 0, st>>>(c_ptr, c_col, c_val, n_rows, n_mids,
                                       reinterpret_cast<unsigned long long*>(s), 0, nullptr);
  }
  DPS_LAUNCHED();
  return DPS_OK;
}

int dps_row_work(const int64_t* c_ptr, const int32_t* c_col, int64_t n_rows, int64_t n_mids,
                 uint32_t* col_count_ws, int64_t* terms, void* stream) {
  DPS_REQUIRE(n_rows >= 0 && n_mids >= 0, DPS_ERR_INVALID, "negative size");
  DPS_REQUIRE(c_ptr && terms && (n_mids == 0 || col_count_ws), DPS_ERR_INVALID, "null array");
  auto st = static_cast<hipStream_t>(stream);
  if (n_rows == 0) return DPS_OK;
  if (n_mids > 0) {
    DPS_HIP_RET(hipMemsetAsync(col_count_ws, 0, n_mids * sizeof(uint32_t), st));
    const unsigned ny = static_cast<unsigned>((n_mids + kColLds - 1) / kColLds);
    k_col_counts<<<dim3(ny > 1 ? 128 : 256, ny), kBlock, 0, st>>>(c_ptr, c_col, n_rows, n_mids,
                                                                  col_count_ws);
    DPS_LAUNCHED();
  }
  k_row_terms<<<grid_for(n_rows, kBlock), kBlock, 0, st>>>(c_ptr, c_col, n_rows, col_count_ws,
                                                          terms);
  DPS_LAUNCHED();
  return DPS_OK;
}

}  // extern "C"
