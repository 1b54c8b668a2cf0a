// Operand layout for the hot kernel (dps_cct.hip) and the single-source
// helpers of the reference-compatible class:
//   dps_target_order   targets relabeled in ascending global walk g (stable
//                      LSD radix sort) -- a pure layout choice;
//   dps_ct_tiles_build C^T cut into target tiles of W = 2^shift labels,
//                      buckets [v][t], zero-padded to 16 bytes; per-bucket max
//                      C and per-tile min g for the hot kernel's bounds.
//                      Entries: W <= 8192 -> packed uint16 (l << 3) | e, l =
//                      label - t*W, one piece of value 2^e: C[y,v] is split
//                      into power-of-two pieces (e <= 7; e <= 5 when l % 4 == 3,
//                      since e = 6, 7 with l % 4 == 3 are the padding codes) --
//                      the kernel's adds are linear in C, so the pieces sum
//                      exactly; W = 16384 -> packed uint16 (l << 2) | e, the
//                      same scheme for packed 4-bit counters (e <= 3; e <= 1
//                      when l % 8 == 7, whose e = 2, 3 are the padding codes);
//                      wider tiles -> packed uint32 (C[y,v] << 16) | (label - t*W);
//   dps_walk_row / dps_row_scores / dps_pair_count: one source row, as the
//                      reference's run() loop computes it (:30-52).
#include "dps_common.hpp"

#include <cstdlib>

namespace dps {
namespace {

constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;

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

constexpr int64_t kTileGminLds = 4096;   // tiles whose g minimum is reduced in LDS

// Entry formats (see the file header), by tile width:
//  kFmtU8  (shift <= 13): uint16 (l << 3) | e adds C[x,v] * 2^e to target l: in
//          the hot kernel's packed-u8 accumulators that is C[x,v] << (8*(l % 4)
//          + e) -- the entry's low five bits ARE the shift.  Codes e = 6, 7 at
//          l % 4 == 3 are reserved for padding (real pieces there stop at 2^5):
//          a bucket's padding is groups of {2^7, 2^7} or {2^7, 2^6, 2^6} on one
//          dword, each adding C[x,v] * 2^32 == 0 to it, so padding needs no
//          multiply by a zero count.
//  kFmtU4  (shift == 14): uint16 (l << 2) | e, the same for packed 4-bit
//          counters: C[x,v] << (4*(l % 8) + e) is again the low five bits; codes
//          e = 2, 3 at l % 8 == 7 are the padding groups {2^3, 2^3} / {2^3, 2^2,
//          2^2} (shift 31, 31 / 31, 30, 30), real pieces there stop at 2^1.
//  kFmt32  (shift >= 15): uint32 (C[y,v] << 16) | l.
constexpr int kFmt32 = 0, kFmtU8 = 1, kFmtU4 = 2;
__host__ __device__ __forceinline__ int tile_fmt(int shift) {
  return shift <= 13 ? kFmtU8 : shift == 14 ? kFmtU4 : kFmt32;
}
__device__ __forceinline__ uint32_t ent_lsh(int fmt) { return fmt == kFmtU8 ? 3u : 2u; }
__device__ __forceinline__ uint32_t ent_max_e(int fmt, uint32_t lab) {
  if (fmt == kFmtU8) return (lab & 3u) == 3u ? 5u : 7u;
  return (lab & 7u) == 7u ? 1u : 3u;
}
__device__ __forceinline__ uint32_t n_pieces(int fmt, uint32_t c, uint32_t lab) {
  if (fmt == kFmt32) return 1u;
  const uint32_t me = ent_max_e(fmt, lab);
  return (c >> me) + static_cast<uint32_t>(__popc(c & ((1u << me) - 1u)));
}
// Bucket size in entries after padding to 16 B (4 uint32 / 8 uint16 entries).
// 16-bit padding comes in groups of two or three entries, so a single padding
// entry is never needed: such a bucket takes nine.
__device__ __forceinline__ uint32_t padded_count(uint32_t tot, uint32_t per16) {
  uint32_t r = (tot + per16 - 1u) & ~(per16 - 1u);
  if (per16 == 8u && r - tot == 1u) r += 8u;
  return r;
}
// Write the entries of (c, local label) at entry index i (16- or 32-bit units).
__device__ __forceinline__ void put_entry(int fmt, uint32_t* ent, int64_t i, uint32_t c,
                                          uint32_t lab) {
  if (fmt == kFmt32) {
    ent[i] = (c << 16) | lab;
    return;
  }
  uint16_t* e16 = reinterpret_cast<uint16_t*>(ent);
  const uint32_t me = ent_max_e(fmt, lab), sh = ent_lsh(fmt);
  for (uint32_t n = c >> me; n > 0; --n) e16[i++] = static_cast<uint16_t>((lab << sh) | me);
  for (uint32_t r = c & ((1u << me) - 1u); r != 0; r &= r - 1u)
    e16[i++] = static_cast<uint16_t>((lab << sh) | static_cast<uint32_t>(__ffs(r) - 1));
}

__global__ __launch_bounds__(kBlock) void k_tile_count(const int64_t* __restrict__ c_ptr,
                                                       const int32_t* __restrict__ c_col,
                                                       const int32_t* __restrict__ c_val,
                                                       const int32_t* __restrict__ rank,
                                                       const int64_t* __restrict__ g,
                                                       int64_t n_rows, TileDim td, int64_t T,
                                                       uint32_t* __restrict__ cnt,
                                                       uint32_t* __restrict__ maxc,
                                                       unsigned long long* __restrict__ gmin,
                                                       int32_t* __restrict__ status) {
  // per-block minimum g of each tile in LDS (one global atomicMin per tile and
  // block instead of one per row onto T hot addresses) when T fits
  __shared__ unsigned long long gmin_s[kTileGminLds];
  const bool lds_gmin = gmin && T <= kTileGminLds;
  if (lds_gmin)
    for (int64_t i = threadIdx.x; i < T; i += kBlock) gmin_s[i] = ~0ull;
  __syncthreads();
  const int lane = lane_id();
  const int64_t wave0 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWavesPerBlock;
  for (int64_t y = wave0; y < n_rows; y += nwaves) {
    const int64_t t = td.tile(label_of(rank, y));
    if (lane == 0 && gmin) {
      if (lds_gmin) atomicMin(&gmin_s[t], static_cast<unsigned long long>(g[y]));
      else atomicMin(&gmin[t], static_cast<unsigned long long>(g[y]));
    }
    for (int64_t j = c_ptr[y] + lane; j < c_ptr[y + 1]; j += kWave) {
      const int32_t c = c_val[j];
      if (c > 0xFFFF && status) *status = DPS_ERR_OVERFLOW;
      const int64_t b = static_cast<int64_t>(c_col[j]) * T + t;
      atomicAdd(&cnt[b], n_pieces(tile_fmt(td.shift), static_cast<uint32_t>(c),
                                  td.local(label_of(rank, y))));
      // C = 1 (most entries when buckets are sparse) needs no atomic: k_round4
      // raises the maximum of every non-empty bucket to at least 1
      if (maxc && c > 1) atomicMax(&maxc[b], static_cast<uint32_t>(c));
    }
  }
  __syncthreads();
  if (lds_gmin)
    for (int64_t i = threadIdx.x; i < T; i += kBlock)
      if (gmin_s[i] != ~0ull) atomicMin(&gmin[i], gmin_s[i]);
}

// Buckets are padded to 16 B (4 uint32 or 8 uint16 entries) so the hot
// kernel's 16-byte chunks never straddle two buckets; padding entries have C = 0.
__global__ __launch_bounds__(kBlock) void k_round4(uint32_t* __restrict__ cnt, int64_t n,
                                                   uint32_t per16, uint32_t* __restrict__ maxc) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * kBlock) {
    const uint32_t c = cnt[i];
    cnt[i] = padded_count(c, per16);
    if (maxc && c > 0 && maxc[i] == 0) maxc[i] = 1;
  }
}

// Padding entries i0 .. i0 + np of a bucket: C = 0 (they add nothing) and a
// label that walks over the tile's dwords, so the hot kernel's branch-free u8
// adds of padding do not pile onto one LDS bank.
__device__ __forceinline__ void pad_bucket(int64_t i0, int64_t np, uint32_t lab_mask, int fmt,
                                           uint32_t* __restrict__ ent) {
  for (int64_t k = 0; k < np; ++k) {
    const int64_t i = i0 + k;
    if (fmt == kFmt32) {
      ent[i] = (static_cast<uint32_t>(i) << 2) & lab_mask & ~3u;
      continue;
    }
    // groups on one dword: {hi, lo, lo} first when the count is odd, then
    // {hi, hi}; hi / lo = 7 / 6 (u8 counters, label % 4 == 3) or 3 / 2
    // (4-bit counters, label % 8 == 7)
    const bool odd = (np & 1) != 0;
    const int64_t grp = odd ? (k < 3 ? 0 : 1 + (k - 3) / 2) : k / 2;
    const bool u8 = fmt == kFmtU8;
    const uint32_t hi = u8 ? 7u : 3u;
    const uint32_t e = (odd && (k == 1 || k == 2)) ? hi - 1u : hi;
    const uint32_t lab = u8 ? (((static_cast<uint32_t>(i0 + 2 * grp) << 2) & lab_mask & ~3u) | 3u)
                            : (((static_cast<uint32_t>(i0 + 2 * grp) << 3) & lab_mask & ~7u) | 7u);
    reinterpret_cast<uint16_t*>(ent)[i] = static_cast<uint16_t>((lab << ent_lsh(fmt)) | e);
  }
}

__global__ __launch_bounds__(kBlock) void k_tile_pad(const int64_t* __restrict__ off, int P,
                                                     const uint32_t* __restrict__ cursor,
                                                     int64_t n, uint32_t lab_mask, int fmt,
                                                     uint32_t* __restrict__ ent) {
  // Bucket b spans off[b*P] .. off[(b+1)*P) (P parts per bucket), its first
  // cursor[b] entries are real.
  for (int64_t b = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; b < n;
       b += static_cast<int64_t>(gridDim.x) * kBlock) {
    const int64_t i0 = off[b * P] + cursor[b];
    pad_bucket(i0, off[(b + 1) * P] - i0, lab_mask, fmt, ent);
  }
}

// Bank order of a bucket's 16-bit entries (both formats: the entry's target
// dword in the hot kernel's accumulator is entry >> 5, its LDS bank for the
// 32-lane groups of ds_add_u32 that dword mod 32).  Lane i of a chunk load
// takes chunk q0 + i, so one scatter instruction adds slot p of 64 consecutive
// chunks; with the build's (label-ordered) layout those hit a few banks many
// times.  Here the bucket is sorted by bank and dealt out so that slot p of
// chunk j holds sorted entry 8 t + p with t = j K mod m (m chunks, K ~ m / 32
// coprime to m): any 32 consecutive chunks of the bucket then cover the bank
// range once per slot.  A permutation inside a bucket only: the adds are the
// same, the sums are the same.  One wave per bucket; buckets above
// kBankMaxEnt entries keep their order.
constexpr int kBankMaxEnt = 8192;
__device__ __forceinline__ int64_t inv_mod(int64_t a, int64_t m) {   // gcd(a, m) == 1
  int64_t t = 0, nt = 1, r = m, nr = a;
  while (nr != 0) {
    const int64_t q = r / nr;
    int64_t x = t - q * nt; t = nt; nt = x;
    x = r - q * nr; r = nr; nr = x;
  }
  return t < 0 ? t + m : t;
}
__device__ __forceinline__ int64_t gcd64(int64_t a, int64_t b) {
  while (b) { const int64_t r = a % b; a = b; b = r; }
  return a;
}
__global__ __launch_bounds__(kWave) void k_tile_bank_order(const uint32_t* __restrict__ off,
                                                           int64_t nb, uint32_t* __restrict__ ent) {
  __shared__ uint16_t src[kBankMaxEnt];
  __shared__ uint32_t hist[32], cur[32];
  const int lane = lane_id();
  uint16_t* e16 = reinterpret_cast<uint16_t*>(ent);
  for (int64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const int64_t w0 = off[b], w1 = off[b + 1];
    const int64_t n = 2 * (w1 - w0);                 // entries, a multiple of 8
    if (n <= 8 || n > kBankMaxEnt) continue;         // one chunk, or too large
    const int64_t m = n >> 3;
    if (lane < 32) hist[lane] = 0;
    __builtin_amdgcn_wave_barrier();
    for (int64_t i = lane; i < n; i += kWave) {
      const uint16_t e = e16[2 * w0 + i];
      src[i] = e;
      atomicAdd(&hist[(e >> 5) & 31u], 1u);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (lane < 32) {
      const uint32_t h = hist[lane];
      uint32_t inc = h;
      for (int d = 1; d < 32; d <<= 1) {
        const uint32_t o = static_cast<uint32_t>(__shfl_up(static_cast<int>(inc), d, 32));
        if (lane >= d) inc += o;
      }
      cur[lane] = inc - h;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    int64_t K = m / 32 > 1 ? m / 32 : 1;
    while (gcd64(K, m) != 1) ++K;
    const int64_t Kinv = inv_mod(K % m, m);
    for (int64_t i = lane; i < n; i += kWave) {
      const uint16_t e = src[i];
      const int64_t si = atomicAdd(&cur[(e >> 5) & 31u], 1u);   // sorted index
      const int64_t t = si >> 3, p = si & 7;
      const int64_t j = m == 1 ? 0 : (t * Kinv) % m;           // t = j K mod m
      e16[2 * w0 + 8 * j + p] = e;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
}

// tile_off in uint32 words (16-bit entries: entry offset / 2, always even).
__global__ __launch_bounds__(kBlock) void k_tile_off32(const int64_t* __restrict__ p64, int P,
                                                       int64_t n, int wshift,
                                                       uint32_t* __restrict__ p32) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i <= n;
       i += static_cast<int64_t>(gridDim.x) * kBlock)
    p32[i] = static_cast<uint32_t>(p64[i * P] >> wshift);
}

__global__ __launch_bounds__(kBlock) void k_tile_scatter(const int64_t* __restrict__ c_ptr,
                                                         const int32_t* __restrict__ c_col,
                                                         const int32_t* __restrict__ c_val,
                                                         const int32_t* __restrict__ rank,
                                                         int64_t n_rows, TileDim td, int64_t T,
                                                         const int64_t* __restrict__ off,
                                                         uint32_t* __restrict__ cursor,
                                                         uint32_t* __restrict__ ent) {
  const int lane = lane_id();
  const int64_t wave0 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWavesPerBlock;
  for (int64_t y = wave0; y < n_rows; y += nwaves) {
    const int64_t lab = label_of(rank, y);
    const int64_t t = td.tile(lab);
    for (int64_t j = c_ptr[y] + lane; j < c_ptr[y + 1]; j += kWave) {
      const int64_t b = static_cast<int64_t>(c_col[j]) * T + t;
      const uint32_t c = static_cast<uint32_t>(c_val[j]);
      const int fmt = tile_fmt(td.shift);
      const uint32_t l = td.local(lab);
      const uint32_t pos = atomicAdd(&cursor[b], n_pieces(fmt, c, l));
      put_entry(fmt, ent, off[b] + pos, c, l);
    }
  }
}

// --------------------------------------------------------------------------
// Block-local tile build (kBlkMids mids per block; more mids take one block per
// mid range, MidRange below): a block owns a contiguous range
// of kBlkLabels target labels -- all inside one tile -- and counts its entries
// per venue in LDS, so the hot buckets of heavy venues take one global atomic
// per block instead of one per entry.  The scatter pass reserves each venue's
// range with one global atomicAdd per (block, venue) and places entries with
// LDS cursors.  Entry order inside a bucket is unspecified either way.
constexpr int kBlkMids = 8192;
constexpr int kBlkLabels = 4096;   // default labels per block (tools/build_ab.py: 1.08 ms vs 1.24 ms at 1024)
// 16 waves per block (one 64-label group each): with 64 KB of LDS per block a
// CU holds two blocks = 32 waves, enough to cover the latency of the gathers.
constexpr int kBlkThreads = 1024;
constexpr int kBlkSub = 8;         // sub-blocks per part

__global__ __launch_bounds__(kBlock) void k_tile_invert(const int32_t* __restrict__ rank,
                                                        int64_t n, int32_t* __restrict__ perm) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * kBlock)
    perm[rank[i]] = static_cast<int32_t>(i);
}

__device__ __forceinline__ int64_t row_of_label(const int32_t* perm, int64_t lab) {
  return perm ? static_cast<int64_t>(perm[lab]) : lab;
}

// A part (labels_per_block consecutive labels of one tile) is processed by S
// sub-blocks, each taking an equal share of the part's entries, so the tail
// part of the highest-g labels -- 8x the mean part's entries, on config3 --
// no longer sets the kernel time.  A sub-block stages, per label of the part,
// the exclusive prefix of its row lengths and the row's C offset minus that
// prefix, then walks its entry range in 64-entry strips with lane = entry:
// the loads are coalesced, and the LDS atomics of a strip mostly hit distinct
// venues (the entries of one C row are distinct venues), where per-thread runs
// through different rows would pile onto the heavy venues' counters.
struct BlockRows {
  uint32_t* rel;   // [nl + 1] exclusive prefix of row lengths (LDS)
  int64_t* d;      // [nl] c_ptr[y] - rel[i] (LDS): entry e of label i is C entry d[i] + e
};

// Stage labels [l0, l1) of the part; returns the part's entry count.  The
// caller provides LDS for kBlkLabels labels.  g != nullptr: also reduce the
// part's smallest g into *gmin_s.
__device__ __forceinline__ uint32_t stage_rows(const int64_t* __restrict__ c_ptr,
                                               const int32_t* __restrict__ perm,
                                               const int64_t* __restrict__ g, int64_t l0,
                                               int64_t l1, BlockRows R, uint32_t* wsum,
                                               unsigned long long* gmin_s) {
  const int nl = static_cast<int>(l1 - l0);
  const int lane = lane_id();
  const int wave = threadIdx.x / kWave;
  constexpr int kWaves = kBlkThreads / kWave;
  // pass 1: row lengths (kept in rel[i + 1]) and row offsets
  unsigned long long gm = ~0ull;
  constexpr int kPer = kBlkLabels / kBlkThreads;   // labels per thread, loads in flight together
  int64_t y[kPer];
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int i = static_cast<int>(threadIdx.x) + u * kBlkThreads;
    y[u] = i < nl ? row_of_label(perm, l0 + i) : -1;
  }
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int i = static_cast<int>(threadIdx.x) + u * kBlkThreads;
    if (y[u] < 0) continue;
    const int64_t beg = c_ptr[y[u]];
    R.rel[i + 1] = static_cast<uint32_t>(c_ptr[y[u] + 1] - beg);
    R.d[i] = beg;
    if (g) gm = min(gm, static_cast<unsigned long long>(g[y[u]]));
  }
  if (g) {
    gm = wave_min(gm);
    if (lane == 0 && gm != ~0ull) atomicMin(gmin_s, gm);
  }
  if (threadIdx.x == 0) R.rel[0] = 0;
  __syncthreads();
  // pass 2: block-wide inclusive scan of rel[1..nl] in strips of kBlkThreads
  uint32_t carry = 0;
  for (int i0 = 0; i0 < nl; i0 += kBlkThreads) {
    const int i = i0 + static_cast<int>(threadIdx.x);
    const uint32_t v = i < nl ? R.rel[i + 1] : 0u;
    const uint32_t inc = wave_inclusive_sum(v);
    if (lane == kWave - 1) wsum[wave] = inc;
    __syncthreads();
    uint32_t off = carry, tot = carry;
    for (int w = 0; w < kWaves; ++w) {
      const uint32_t ws = wsum[w];
      off += w < wave ? ws : 0u;
      tot += ws;
    }
    if (i < nl) {
      R.rel[i + 1] = off + inc;
      R.d[i] -= static_cast<int64_t>(off + inc - v);
    }
    carry = tot;
    __syncthreads();
  }
  return carry;
}

// Strip table of a sub-block: strip k covers entries [e0 + 64k, e0 + 64k + 64)
// of the part; tab[k] = the label holding its first entry, tab[ns] = the label
// holding entry e1 - 1, so strip k's labels lie in [tab[k], tab[k + 1]].
// Built by one pass over the labels (each writes the strip starts it holds).
constexpr int kMaxStrips = 1024;

__device__ __forceinline__ void strip_table(const BlockRows& R, int nl, uint32_t e0, uint32_t e1,
                                            int* tab) {
  const uint32_t ns = (e1 - e0 + kWave - 1) / kWave;
  for (int i = threadIdx.x; i < nl; i += kBlkThreads) {
    const uint32_t a = max(R.rel[i], e0), b = min(R.rel[i + 1], e1);
    if (a >= b) continue;
    for (uint32_t k = (a - e0 + kWave - 1) / kWave; k < ns && e0 + k * kWave < b; ++k) tab[k] = i;
    if (e1 - 1 >= a && e1 - 1 < b) tab[ns] = i;
  }
  __syncthreads();
}

// Last label i in [lo, hi] with rel[i] <= e.
__device__ __forceinline__ int label_at(const uint32_t* rel, int lo, int hi, uint32_t e) {
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (rel[mid] <= e) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// Visit entries [e0, e1) of the staged labels in 64-entry strips, lane =
// entry, kStripU strips per wave at a time (their loads in flight together):
// fn(label index, venue, C).  A strip's label window comes from the strip
// table (or, past its capacity, from two wave-uniform searches); each lane then
// searches only inside it.
constexpr int kStripU = 4;

template <typename Fn>
__device__ __forceinline__ void walk_strips(const BlockRows& R, int nl, uint32_t e0, uint32_t e1,
                                            const int* tab, const int32_t* __restrict__ c_col,
                                            const int32_t* __restrict__ c_val, Fn&& fn) {
  const int lane = lane_id();
  constexpr uint32_t kWaves = kBlkThreads / kWave;
  const uint32_t ns = (e1 - e0 + kWave - 1) / kWave;
  for (uint32_t k0 = threadIdx.x / kWave; k0 < ns; k0 += kWaves * kStripU) {
    int li[kStripU];
    int64_t j[kStripU];
#pragma unroll
    for (int u = 0; u < kStripU; ++u) {
      const uint32_t k = k0 + u * kWaves;
      li[u] = -1;
      j[u] = 0;
      if (k >= ns) continue;                      // wave-uniform
      const uint32_t s = e0 + k * kWave;
      int lo, hi;
      if (ns <= kMaxStrips) {
        lo = tab[k];
        hi = tab[k + 1];
      } else {
        lo = label_at(R.rel, 0, nl - 1, s);
        hi = label_at(R.rel, lo, nl - 1, min(s + kWave - 1u, e1 - 1u));
      }
      const uint32_t e = s + static_cast<uint32_t>(lane);
      if (e < e1) {
        li[u] = label_at(R.rel, lo, hi, e);
        j[u] = R.d[li[u]] + e;
      }
    }
    int32_t v[kStripU], c[kStripU];
#pragma unroll
    for (int u = 0; u < kStripU; ++u) {
      v[u] = li[u] >= 0 ? c_col[j[u]] : 0;
      c[u] = li[u] >= 0 ? c_val[j[u]] : 0;
    }
#pragma unroll
    for (int u = 0; u < kStripU; ++u)
      if (li[u] >= 0) fn(li[u], v[u], c[u]);
  }
}

// perm = inverse of rank, and in the same pass over the rows (coalesced row
// offsets) the entries per part, reduced in an LDS histogram per block (one
// global atomic per part and block); n_parts <= kPartLds.
constexpr int kPartLds = 8192;
__global__ __launch_bounds__(kBlock) void k_invert_and_parts(const int32_t* __restrict__ rank,
                                                             const int64_t* __restrict__ c_ptr,
                                                             int64_t n, int labels_per_block,
                                                             int n_parts, int32_t* __restrict__ perm,
                                                             uint32_t* __restrict__ part_n) {
  __shared__ uint32_t h[kPartLds];
  for (int i = threadIdx.x; i < n_parts; i += kBlock) h[i] = 0;
  __syncthreads();
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * kBlock) {
    const int64_t lab = rank ? static_cast<int64_t>(rank[i]) : i;
    if (rank) perm[lab] = static_cast<int32_t>(i);
    const uint32_t len = static_cast<uint32_t>(c_ptr[i + 1] - c_ptr[i]);
    if (len) atomicAdd(&h[lab / labels_per_block], len);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n_parts; i += kBlock)
    if (h[i]) atomicAdd(&part_n[i], h[i]);
}

// Entries per part (sum of its labels' row lengths), one atomic per wave.
__global__ __launch_bounds__(kBlock) void k_part_entries(const int64_t* __restrict__ c_ptr,
                                                         const int32_t* __restrict__ perm,
                                                         int64_t n_targets, int labels_per_block,
                                                         uint32_t* __restrict__ part_n) {
  const int64_t wave0 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWavesPerBlock;
  for (int64_t l0 = wave0 * kWave; l0 < n_targets; l0 += nwaves * kWave) {
    const int64_t l = l0 + lane_id();
    uint32_t len = 0;
    if (l < n_targets) {
      const int64_t y = row_of_label(perm, l);
      len = static_cast<uint32_t>(c_ptr[y + 1] - c_ptr[y]);
    }
    const uint32_t tot = static_cast<uint32_t>(readlane(static_cast<int>(wave_inclusive_sum(len)), kWave - 1));
    if (lane_id() == 0 && tot) atomicAdd(&part_n[l0 / labels_per_block], tot);
  }
}

// Sub-block sb of a part with n entries: its share [e0, e1) and the part's
// number of active sub-blocks (n / kSubEntries, at least 1, at most S).
constexpr uint32_t kSubEntries = 32768;
struct SubRange {
  uint32_t e0, e1;
  int n_sub;
};
__device__ __forceinline__ SubRange sub_range(uint32_t n, uint32_t sb, int S) {
  int n_sub = static_cast<int>((n + kSubEntries - 1) / kSubEntries);
  n_sub = n_sub < 1 ? 1 : n_sub > S ? S : n_sub;
  SubRange r;
  r.n_sub = n_sub;
  r.e0 = static_cast<uint32_t>(static_cast<uint64_t>(n) * sb / n_sub);
  r.e1 = static_cast<uint32_t>(static_cast<uint64_t>(n) * (sb + 1) / n_sub);
  return r;
}

// Mid range r of the block-local build: mids [m0, m0 + n), n <= kBlkMids (the
// LDS counters of one block); a build over more mids launches one block per
// (part, sub-block, range), each walking the part's entries and keeping its
// range's.
struct MidRange {
  int64_t m0;
  int n;
};
__device__ __forceinline__ MidRange mid_range(int64_t r, int64_t n_mids) {
  MidRange m;
  m.m0 = r * kBlkMids;
  const int64_t left = n_mids - m.m0;
  m.n = static_cast<int>(left < kBlkMids ? (left > 0 ? left : 0) : kBlkMids);
  return m;
}

// Part p = (t, h) of tile t (labels_per_block labels, P parts per tile),
// sub-block sb of up to S (sub_range: one per kSubEntries entries of the part).
// Counting writes the sub-block's per-venue piece counts and maxima into the
// part's slots cntp/mxp[(v*T + t)*P + h] -- plain stores when the part has one
// active sub-block, one global atomic per (sub-block, venue) otherwise;
// k_tile_parts_fix pads each bucket and reduces the maxima, and one exclusive
// scan over the [v][t][h] order gives every part its base offset.
__global__ __launch_bounds__(kBlkThreads) void k_tile_count_blk(
    const int64_t* __restrict__ c_ptr, const int32_t* __restrict__ c_col,
    const int32_t* __restrict__ c_val, const int32_t* __restrict__ perm,
    const int64_t* __restrict__ g, int64_t n_targets, int64_t n_mids, TileDim td, int64_t T,
    int labels_per_block, int P, int S, int n_ranges, const uint32_t* __restrict__ part_n,
    uint32_t* __restrict__ cntp, uint32_t* __restrict__ mxp,
    unsigned long long* __restrict__ gmin, int32_t* __restrict__ status) {
  __shared__ uint32_t cnt_s[kBlkMids];
  __shared__ uint32_t mx_s[kBlkMids];
  __shared__ uint32_t rel_s[kBlkLabels + 1];
  __shared__ int64_t d_s[kBlkLabels];
  __shared__ int tab_s[kMaxStrips + 1];
  __shared__ uint32_t wsum[kBlkThreads / kWave];
  __shared__ unsigned long long gmin_s;
  __shared__ int ovf_s;
  // sub-block major (block = (range * S + sb) * n_parts + part): the parts'
  // first sub-blocks -- the only ones most parts use -- spread over every XCD
  const int64_t n_parts = gridDim.x / (static_cast<int64_t>(S) * n_ranges);
  const int64_t part = blockIdx.x % n_parts;
  const int64_t q = blockIdx.x / n_parts;
  const uint32_t sb = static_cast<uint32_t>(q % S);
  const MidRange mr = mid_range(q / S, n_mids);
  const SubRange sr = sub_range(part_n[part], sb, S);
  if (static_cast<int>(sb) >= sr.n_sub) return;   // block-uniform: before any barrier
  for (int v = threadIdx.x; v < mr.n; v += kBlkThreads) { cnt_s[v] = 0; mx_s[v] = 0; }
  if (threadIdx.x == 0) { gmin_s = ~0ull; ovf_s = 0; }
  const int fmt = tile_fmt(td.shift);
  const int64_t l0 = part * labels_per_block;
  const int64_t l1 = min(l0 + labels_per_block, n_targets);
  const int64_t t = td.tile(l0);
  const int64_t h = part % P;
  __syncthreads();
  const BlockRows R{rel_s, d_s};
  const int nl = static_cast<int>(l1 - l0);
  const bool do_g = gmin && sb == 0 && mr.m0 == 0;
  [[maybe_unused]] const uint32_t n = stage_rows(c_ptr, perm, do_g ? g : nullptr, l0, l1, R, wsum, &gmin_s);
  DPS_DASSERT(n == part_n[part]);
  if (sr.e1 - sr.e0 <= kMaxStrips * kWave) strip_table(R, nl, sr.e0, sr.e1, tab_s);
  const uint32_t lab0 = static_cast<uint32_t>(l0);
  walk_strips(R, nl, sr.e0, sr.e1, tab_s, c_col, c_val, [&](int i, int32_t v, int32_t c) {
    if (c > 0xFFFF) ovf_s = 1;
    const uint32_t lv = static_cast<uint32_t>(v - mr.m0);
    if (lv >= static_cast<uint32_t>(mr.n)) return;   // another block's mid range
    atomicAdd(&cnt_s[lv], n_pieces(fmt, static_cast<uint32_t>(c), lab0 + static_cast<uint32_t>(i)));
    if (c > 1) atomicMax(&mx_s[lv], static_cast<uint32_t>(c));   // 1 by k_tile_parts_fix
  });
  __syncthreads();
  if (threadIdx.x == 0 && ovf_s && status) *status = DPS_ERR_OVERFLOW;
  for (int lv = threadIdx.x; lv < mr.n; lv += kBlkThreads) {
    if (!cnt_s[lv]) continue;
    const int64_t v = mr.m0 + lv;
    const int64_t slot = (v * T + t) * P + h;
    if (sr.n_sub == 1) {
      cntp[slot] = cnt_s[lv];
      mxp[slot] = mx_s[lv];
    } else {
      atomicAdd(&cntp[slot], cnt_s[lv]);
      if (mx_s[lv]) atomicMax(&mxp[slot], mx_s[lv]);
    }
  }
  if (threadIdx.x == 0 && do_g && gmin_s != ~0ull) atomicMin(&gmin[t], gmin_s);
}

// Per bucket b: tot = real entries (kept in cnt[b] for the padding pass),
// padding to 16 B added to the last part, maxc = max over the parts.
__global__ __launch_bounds__(kBlock) void k_tile_parts_fix(uint32_t* __restrict__ cntp,
                                                           const uint32_t* __restrict__ mxp,
                                                           int64_t nb, int P, uint32_t per16,
                                                           uint32_t* __restrict__ cnt,
                                                           uint32_t* __restrict__ maxc) {
  for (int64_t b = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; b < nb;
       b += static_cast<int64_t>(gridDim.x) * kBlock) {
    uint32_t tot = 0, mx = 0;
    for (int h = 0; h < P; ++h) {
      tot += cntp[b * P + h];
      mx = max(mx, mxp[b * P + h]);
    }
    cnt[b] = tot;
    cntp[b * P + P - 1] += padded_count(tot, per16) - tot;
    if (maxc) maxc[b] = (tot > 0 && mx == 0) ? 1u : mx;   // C = 1 entries skip the max
  }
}

// Scatter: a part with one active sub-block places its entries from the part's
// base offsets; with several, each sub-block counts its own entries per venue,
// reserves its range inside every part slot it touches (one global atomic per
// venue on curp), then places them with 64-bit LDS cursors.
__global__ __launch_bounds__(kBlkThreads) void k_tile_scatter_blk(
    const int64_t* __restrict__ c_ptr, const int32_t* __restrict__ c_col,
    const int32_t* __restrict__ c_val, const int32_t* __restrict__ perm, int64_t n_targets,
    int64_t n_mids, TileDim td, int64_t T, int labels_per_block, int P, int S, int n_ranges,
    const uint32_t* __restrict__ part_n, const int64_t* __restrict__ offp,
    uint32_t* __restrict__ curp, uint32_t* __restrict__ ent) {
  __shared__ uint32_t cnt_s[kBlkMids];
  __shared__ unsigned long long base_s[kBlkMids];
  __shared__ uint32_t rel_s[kBlkLabels + 1];
  __shared__ int64_t d_s[kBlkLabels];
  __shared__ int tab_s[kMaxStrips + 1];
  __shared__ uint32_t wsum[kBlkThreads / kWave];
  // block = (range * S + sb) * n_parts + part, as in k_tile_count_blk
  const int64_t n_parts = gridDim.x / (static_cast<int64_t>(S) * n_ranges);
  const int64_t part = blockIdx.x % n_parts;
  const int64_t q = blockIdx.x / n_parts;
  const uint32_t sb = static_cast<uint32_t>(q % S);
  const MidRange mr = mid_range(q / S, n_mids);
  const SubRange sr = sub_range(part_n[part], sb, S);
  if (static_cast<int>(sb) >= sr.n_sub) return;   // block-uniform: before any barrier
  for (int v = threadIdx.x; v < mr.n; v += kBlkThreads) cnt_s[v] = 0;
  const int fmt = tile_fmt(td.shift);
  const int64_t l0 = part * labels_per_block;
  const int64_t l1 = min(l0 + labels_per_block, n_targets);
  const int64_t t = td.tile(l0);
  const int64_t h = part % P;
  __syncthreads();
  const BlockRows R{rel_s, d_s};
  const int nl = static_cast<int>(l1 - l0);
  stage_rows(c_ptr, perm, nullptr, l0, l1, R, wsum, nullptr);
  if (sr.e1 - sr.e0 <= kMaxStrips * kWave) strip_table(R, nl, sr.e0, sr.e1, tab_s);
  const uint32_t lab0 = td.local(l0);   // (a part lies inside one tile)
  if (sr.n_sub == 1) {
    for (int lv = threadIdx.x; lv < mr.n; lv += kBlkThreads)
      base_s[lv] = static_cast<unsigned long long>(offp[((mr.m0 + lv) * T + t) * P + h]);
  } else {
    walk_strips(R, nl, sr.e0, sr.e1, tab_s, c_col, c_val, [&](int i, int32_t v, int32_t c) {
      const uint32_t lv = static_cast<uint32_t>(v - mr.m0);
      if (lv >= static_cast<uint32_t>(mr.n)) return;
      atomicAdd(&cnt_s[lv], n_pieces(fmt, static_cast<uint32_t>(c), lab0 + static_cast<uint32_t>(i)));
    });
    __syncthreads();
    for (int lv = threadIdx.x; lv < mr.n; lv += kBlkThreads) {
      const uint32_t nv = cnt_s[lv];
      if (!nv) continue;
      const int64_t slot = ((mr.m0 + lv) * T + t) * P + h;
      base_s[lv] = static_cast<unsigned long long>(offp[slot] + atomicAdd(&curp[slot], nv));
    }
  }
  __syncthreads();
  walk_strips(R, nl, sr.e0, sr.e1, tab_s, c_col, c_val, [&](int i, int32_t v, int32_t c) {
    const uint32_t lv = static_cast<uint32_t>(v - mr.m0);
    if (lv >= static_cast<uint32_t>(mr.n)) return;
    const uint32_t lab = lab0 + static_cast<uint32_t>(i);
    const unsigned long long pos =
        atomicAdd(&base_s[lv], static_cast<unsigned long long>(
                                  n_pieces(fmt, static_cast<uint32_t>(c), lab)));
    put_entry(fmt, ent, static_cast<int64_t>(pos), static_cast<uint32_t>(c), lab);
  });
}

// --------------------------------------------------------------------------
// Both tile sets of the bench shape in one walk of C (round 6):
// the 4-bit tiles A (16384 / 15360 targets) and their companion u8 half tiles
// B (8192 / 7680).  A part (lpb labels) lies inside one tile of each set, so a
// block stages its labels and walks its entries once and counts -- then places
// -- every entry in both formats; the per-(venue, part) maximum is shared (the
// same C values).  Count LDS: two count arrays and one maximum, 96 KiB + the
// staged rows; scatter: two 32-bit cursor arrays (the host checks both sets'
// entries fit 32 bits).
__global__ __launch_bounds__(kBlkThreads) void k_tile_count_dual(
    const int64_t* __restrict__ c_ptr, const int32_t* __restrict__ c_col,
    const int32_t* __restrict__ c_val, const int32_t* __restrict__ perm,
    const int64_t* __restrict__ g, int64_t n_targets, int64_t n_mids, TileDim tdA, int64_t TA,
    TileDim tdB, int64_t TB, int labels_per_block, int PA, int PB, int S, int n_ranges,
    const uint32_t* __restrict__ part_n, uint32_t* __restrict__ cntpA, uint32_t* __restrict__ mxpA,
    uint32_t* __restrict__ cntpB, uint32_t* __restrict__ mxpB,
    unsigned long long* __restrict__ gmin, int32_t* __restrict__ status,
    const int32_t* __restrict__ hv_slot, int n_hv, uint16_t* __restrict__ hv_c) {
  __shared__ uint32_t cntA_s[kBlkMids];
  __shared__ uint32_t cntB_s[kBlkMids];
  __shared__ uint32_t mx_s[kBlkMids];
  __shared__ uint32_t rel_s[kBlkLabels + 1];
  __shared__ int64_t d_s[kBlkLabels];
  __shared__ int tab_s[kMaxStrips + 1];
  __shared__ uint32_t wsum[kBlkThreads / kWave];
  __shared__ unsigned long long gmin_s;
  __shared__ int ovf_s;
  const int64_t n_parts = gridDim.x / (static_cast<int64_t>(S) * n_ranges);
  const int64_t part = blockIdx.x % n_parts;
  const int64_t q = blockIdx.x / n_parts;
  const uint32_t sb = static_cast<uint32_t>(q % S);
  const MidRange mr = mid_range(q / S, n_mids);
  const SubRange sr = sub_range(part_n[part], sb, S);
  if (static_cast<int>(sb) >= sr.n_sub) return;   // block-uniform: before any barrier
  for (int v = threadIdx.x; v < mr.n; v += kBlkThreads) { cntA_s[v] = 0; cntB_s[v] = 0; mx_s[v] = 0; }
  if (threadIdx.x == 0) { gmin_s = ~0ull; ovf_s = 0; }
  const int fmtA = tile_fmt(tdA.shift), fmtB = tile_fmt(tdB.shift);
  const int64_t l0 = part * labels_per_block;
  const int64_t l1 = min(l0 + labels_per_block, n_targets);
  const int64_t tA = tdA.tile(l0), tB = tdB.tile(l0);
  const int64_t hA = part % PA, hB = part % PB;
  __syncthreads();
  const BlockRows R{rel_s, d_s};
  const int nl = static_cast<int>(l1 - l0);
  const bool do_g = gmin && sb == 0 && mr.m0 == 0;
  stage_rows(c_ptr, perm, do_g ? g : nullptr, l0, l1, R, wsum, &gmin_s);
  if (sr.e1 - sr.e0 <= kMaxStrips * kWave) strip_table(R, nl, sr.e0, sr.e1, tab_s);
  const uint32_t lab0 = static_cast<uint32_t>(l0);   // (the pieces depend on label % 8 only)
  walk_strips(R, nl, sr.e0, sr.e1, tab_s, c_col, c_val, [&](int i, int32_t v, int32_t c) {
    if (c > 0xFFFF) ovf_s = 1;
    const uint32_t lv = static_cast<uint32_t>(v - mr.m0);
    if (lv >= static_cast<uint32_t>(mr.n)) return;
    const uint32_t lab = lab0 + static_cast<uint32_t>(i);
    atomicAdd(&cntA_s[lv], n_pieces(fmtA, static_cast<uint32_t>(c), lab));
    atomicAdd(&cntB_s[lv], n_pieces(fmtB, static_cast<uint32_t>(c), lab));
    if (c > 1) atomicMax(&mx_s[lv], static_cast<uint32_t>(c));
    if (hv_c) {   // the heavy-venue table (dps_heavy_table's layout), same walk
      const int sl = hv_slot[v];
      if (sl >= 0) hv_c[static_cast<int64_t>(lab) * n_hv + sl] = static_cast<uint16_t>(c < 0xFFFF ? c : 0xFFFF);
    }
  });
  __syncthreads();
  if (threadIdx.x == 0 && ovf_s && status) *status = DPS_ERR_OVERFLOW;
  for (int lv = threadIdx.x; lv < mr.n; lv += kBlkThreads) {
    if (!cntA_s[lv]) continue;
    const int64_t v = mr.m0 + lv;
    const int64_t sa = (v * TA + tA) * PA + hA, sbb = (v * TB + tB) * PB + hB;
    if (sr.n_sub == 1) {
      cntpA[sa] = cntA_s[lv];
      mxpA[sa] = mx_s[lv];
      cntpB[sbb] = cntB_s[lv];
      mxpB[sbb] = mx_s[lv];
    } else {
      atomicAdd(&cntpA[sa], cntA_s[lv]);
      atomicAdd(&cntpB[sbb], cntB_s[lv]);
      if (mx_s[lv]) {
        atomicMax(&mxpA[sa], mx_s[lv]);
        atomicMax(&mxpB[sbb], mx_s[lv]);
      }
    }
  }
  if (threadIdx.x == 0 && do_g && gmin_s != ~0ull) atomicMin(&gmin[tA], gmin_s);
}

__global__ __launch_bounds__(kBlkThreads) void k_tile_scatter_dual(
    const int64_t* __restrict__ c_ptr, const int32_t* __restrict__ c_col,
    const int32_t* __restrict__ c_val, const int32_t* __restrict__ perm, int64_t n_targets,
    int64_t n_mids, TileDim tdA, int64_t TA, TileDim tdB, int64_t TB, int labels_per_block, int PA,
    int PB, int S, int n_ranges, const uint32_t* __restrict__ part_n,
    const int64_t* __restrict__ offpA, uint32_t* __restrict__ curpA, uint32_t* __restrict__ entA,
    const int64_t* __restrict__ offpB, uint32_t* __restrict__ curpB, uint32_t* __restrict__ entB) {
  __shared__ uint32_t baseA_s[kBlkMids];   // counts, then 32-bit entry cursors
  __shared__ uint32_t baseB_s[kBlkMids];
  __shared__ uint32_t rel_s[kBlkLabels + 1];
  __shared__ int64_t d_s[kBlkLabels];
  __shared__ int tab_s[kMaxStrips + 1];
  __shared__ uint32_t wsum[kBlkThreads / kWave];
  const int64_t n_parts = gridDim.x / (static_cast<int64_t>(S) * n_ranges);
  const int64_t part = blockIdx.x % n_parts;
  const int64_t q = blockIdx.x / n_parts;
  const uint32_t sb = static_cast<uint32_t>(q % S);
  const MidRange mr = mid_range(q / S, n_mids);
  const SubRange sr = sub_range(part_n[part], sb, S);
  if (static_cast<int>(sb) >= sr.n_sub) return;   // block-uniform: before any barrier
  for (int v = threadIdx.x; v < mr.n; v += kBlkThreads) { baseA_s[v] = 0; baseB_s[v] = 0; }
  const int fmtA = tile_fmt(tdA.shift), fmtB = tile_fmt(tdB.shift);
  const int64_t l0 = part * labels_per_block;
  const int64_t l1 = min(l0 + labels_per_block, n_targets);
  const int64_t tA = tdA.tile(l0), tB = tdB.tile(l0);
  const int64_t hA = part % PA, hB = part % PB;
  __syncthreads();
  const BlockRows R{rel_s, d_s};
  const int nl = static_cast<int>(l1 - l0);
  stage_rows(c_ptr, perm, nullptr, l0, l1, R, wsum, nullptr);
  if (sr.e1 - sr.e0 <= kMaxStrips * kWave) strip_table(R, nl, sr.e0, sr.e1, tab_s);
  const uint32_t labA0 = tdA.local(l0), labB0 = tdB.local(l0);   // (a part lies in one tile)
  if (sr.n_sub == 1) {
    for (int lv = threadIdx.x; lv < mr.n; lv += kBlkThreads) {
      baseA_s[lv] = static_cast<uint32_t>(offpA[((mr.m0 + lv) * TA + tA) * PA + hA]);
      baseB_s[lv] = static_cast<uint32_t>(offpB[((mr.m0 + lv) * TB + tB) * PB + hB]);
    }
  } else {
    walk_strips(R, nl, sr.e0, sr.e1, tab_s, c_col, c_val, [&](int i, int32_t v, int32_t c) {
      const uint32_t lv = static_cast<uint32_t>(v - mr.m0);
      if (lv >= static_cast<uint32_t>(mr.n)) return;
      atomicAdd(&baseA_s[lv], n_pieces(fmtA, static_cast<uint32_t>(c), labA0 + static_cast<uint32_t>(i)));
      atomicAdd(&baseB_s[lv], n_pieces(fmtB, static_cast<uint32_t>(c), labB0 + static_cast<uint32_t>(i)));
    });
    __syncthreads();
    for (int lv = threadIdx.x; lv < mr.n; lv += kBlkThreads) {
      const uint32_t na = baseA_s[lv];
      if (!na) continue;
      const int64_t sa = ((mr.m0 + lv) * TA + tA) * PA + hA;
      const int64_t sbb = ((mr.m0 + lv) * TB + tB) * PB + hB;
      baseA_s[lv] = static_cast<uint32_t>(offpA[sa] + atomicAdd(&curpA[sa], na));
      baseB_s[lv] = static_cast<uint32_t>(offpB[sbb] + atomicAdd(&curpB[sbb], baseB_s[lv]));
    }
  }
  __syncthreads();
  walk_strips(R, nl, sr.e0, sr.e1, tab_s, c_col, c_val, [&](int i, int32_t v, int32_t c) {
    const uint32_t lv = static_cast<uint32_t>(v - mr.m0);
    if (lv >= static_cast<uint32_t>(mr.n)) return;
    const uint32_t cu = static_cast<uint32_t>(c);
    const uint32_t la = labA0 + static_cast<uint32_t>(i), lb = labB0 + static_cast<uint32_t>(i);
    const uint32_t pa = atomicAdd(&baseA_s[lv], n_pieces(fmtA, cu, la));
    put_entry(fmtA, entA, static_cast<int64_t>(pa), cu, la);
    const uint32_t pb = atomicAdd(&baseB_s[lv], n_pieces(fmtB, cu, lb));
    put_entry(fmtB, entB, static_cast<int64_t>(pb), cu, lb);
  });
}

// --------------------------------------------------------------------------
// Single-source dense row: one block per target tile; out_m in ORIGINAL order.
__global__ __launch_bounds__(kBlock) void k_walk_row(const int32_t* __restrict__ src_col,
                                                     const int32_t* __restrict__ src_val,
                                                     int64_t src_len, int64_t n_targets, TileDim td,
                                                     int64_t T, const uint32_t* __restrict__ off,
                                                     const uint32_t* __restrict__ ent,
                                                     const int32_t* __restrict__ t_perm,
                                                     int64_t* __restrict__ out_m) {
  // int32 accumulators for up to 32768 labels; wider tiles run in 32768-label parts
  extern __shared__ __attribute__((aligned(16))) int32_t acc[];
  const int W = static_cast<int>(td.w());
  const int P = W < 32768 ? W : 32768;
  const int64_t t = blockIdx.x;
  for (int part = 0; part < W / P; ++part) {
    for (int i = threadIdx.x; i < P; i += kBlock) acc[i] = 0;
    __syncthreads();
    for (int64_t j = 0; j < src_len; ++j) {
      const int64_t b = static_cast<int64_t>(src_col[j]) * T + t;
      const int cx = src_val[j];
      for (uint32_t i = off[b] + threadIdx.x; i < off[b + 1]; i += kBlock) {
        const uint32_t w = ent[i];
        const int fmt = tile_fmt(td.shift);
        if (fmt != kFmt32) {   // two 16-bit entries per word (W = P here)
          const uint32_t sh = ent_lsh(fmt);
#pragma unroll
          for (int half = 0; half < 2; ++half) {
            const uint32_t h = (w >> (16 * half)) & 0xFFFFu;
            const uint32_t e = h & ((1u << sh) - 1u), lab = h >> sh;
            if (e > ent_max_e(fmt, lab)) continue;   // padding
            atomicAdd(&acc[lab], cx << e);
          }
          continue;
        }
        const uint32_t lab = w & 0xFFFFu;
        if (static_cast<int>(lab) / P != part) continue;
        atomicAdd(&acc[lab % P], cx * static_cast<int>(w >> 16));
      }
    }
    __syncthreads();
    const int64_t y0 = t * W + static_cast<int64_t>(part) * P;
    for (int i = threadIdx.x; i < P && y0 + i < n_targets; i += kBlock) {
      const int64_t lab = y0 + i;
      out_m[t_perm ? t_perm[lab] : lab] = acc[i];
    }
    __syncthreads();
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

// Label mask of the padding entries: a power of two minus one that stays
// below the tile width (the padding labels only spread no-op adds over banks).
uint32_t pad_mask(TileDim td) {
  return td.t15 ? (1u << (td.shift - 1)) - 1u : (1u << td.shift) - 1u;
}

// Labels per block of the block-local build: a power of two in [1024, tile_w]
// (DPATHSIM_TILE_LPB overrides the default in the -DDPS_PROFILE build, for A/B runs).  Every block writes
// one count slot per (mid, part), so fewer, wider parts shrink the slot arrays
// and their scan; more parts give more blocks.
int tile_lpb(int32_t tile_w) {
  int lpb = kBlkLabels;
#ifdef DPS_PROFILE
  if (const char* e = std::getenv("DPATHSIM_TILE_LPB")) lpb = std::atoi(e);
#endif
  if (lpb < 1024 || lpb > kBlkLabels || (lpb & (lpb - 1))) lpb = kBlkLabels;
  if (tile_dim(tile_w).t15) return 3840;   // a divisor of 7680 and 15360 (parts never cross tiles)
  return tile_w < lpb ? tile_w : lpb;
}

// Sub-blocks per part of the block-local build (entries split evenly).
int tile_sub() {
  int sub = kBlkSub;
#ifdef DPS_PROFILE
  if (const char* e = std::getenv("DPATHSIM_TILE_SUB")) sub = std::atoi(e);
#endif
  return sub < 1 || sub > 64 ? kBlkSub : sub;
}

// Builds over more than kBlkMids mids: the block-local path with one block
// per mid range reads C once per range, so it is taken up to kMaxMidRanges
// ranges (config5, 20k venues, 3 ranges: 7.1 -> 2.8 ms) and the global-atomic
// counting sort above (config4, 200k topics, 25 ranges: 7.5 vs 13.7 ms);
// DPATHSIM_TILE_GLOBAL=1 / 0 forces one or the other (-DDPS_PROFILE build).
constexpr int64_t kMaxMidRanges = 8;
bool tile_global(int64_t n_mids) {
  if (n_mids <= kBlkMids) return false;
  if (const int t = tuning(DPS_TUNE_TILE_BUILD)) return t == 2;
#ifdef DPS_PROFILE
  if (const char* e = std::getenv("DPATHSIM_TILE_GLOBAL")) return std::atoi(e) != 0;
#endif
  return (n_mids + kBlkMids - 1) / kBlkMids > kMaxMidRanges;
}

// Parts per tile of the block-local build (1 on the global-atomic path).
int64_t tile_parts(int64_t n_mids, int32_t tile_w) {
  if (tile_global(n_mids)) return 1;
  const int lpb = tile_lpb(tile_w);
  return tile_w > lpb ? tile_w / lpb : 1;
}

// The bank-order pass over the finished buckets (16-bit entries only).
int bank_order(bool p16, int64_t nb, const uint32_t* tile_off, uint32_t* tile_ent,
               hipStream_t st) {
  const int t = tuning(DPS_TUNE_BANK_ORDER);
  if (!p16 || nb <= 0 || t != 1) return DPS_OK;
  const int64_t grid = nb < 65536 ? nb : 65536;
  k_tile_bank_order<<<static_cast<unsigned>(grid), kWave, 0, st>>>(tile_off, nb, tile_ent);
  DPS_LAUNCHED();
  return DPS_OK;
}

// Count sums per bucket (dps_ct_tiles_sums): 16 lanes per bucket, a sum of
// the entries' piece values (padding codes add nothing).
__device__ __forceinline__ uint32_t piece_val(int fmt, uint32_t h) {
  const uint32_t e = fmt == kFmtU8 ? (h & 7u) : (h & 3u);
  const uint32_t lab = h >> ent_lsh(fmt);
  return e > ent_max_e(fmt, lab) ? 0u : (1u << e);
}
__global__ __launch_bounds__(kBlock) void k_tile_sums(const uint32_t* __restrict__ off,
                                                      const uint32_t* __restrict__ ent, int64_t nb,
                                                      int fmt, uint32_t* __restrict__ sum) {
  const int sub = threadIdx.x & 15;
  for (int64_t b = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) >> 4; b < nb;
       b += (static_cast<int64_t>(gridDim.x) * kBlock) >> 4) {
    uint32_t s = 0;
    for (uint32_t i = off[b] + sub; i < off[b + 1]; i += 16) {
      const uint32_t w = ent[i];
      s += fmt == kFmt32 ? (w >> 16) : piece_val(fmt, w & 0xFFFFu) + piece_val(fmt, w >> 16);
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 16);
    if (sub == 0) sum[b] = s;
  }
}

// --------------------------------------------------------------------------
// Sorted tile build (dps_ct_tiles_build2, many mids -- config4's 200k topics,
// where the per-entry global atomics on n_mids * T bucket counters cost 5.8
// ms).  The C entries are laid out in target-label order (row y's entries
// at Q[label(y)], Q the scan of the row lengths by label) as pairs
// ((t << 32) | v, (local label << 16) | C); one stable LSD radix sort on the
// mid bits alone then yields (v, label) order, i.e. the (v, t) buckets
// contiguous and each bucket's entries by label.  Buckets are then counted,
// laid out and written from the sorted order -- coalesced, no atomics on the
// 24.6 M bucket counters.  Pairs past nnz (the capacity is a host bound)
// carry the mid n_mids and sort last.
__global__ __launch_bounds__(kBlock) void k_label_len(const int64_t* __restrict__ c_ptr,
                                                      const int32_t* __restrict__ rank,
                                                      int64_t n_rows, uint32_t* __restrict__ len) {
  for (int64_t y = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; y < n_rows;
       y += static_cast<int64_t>(gridDim.x) * kBlock)
    len[label_of(rank, y)] = static_cast<uint32_t>(c_ptr[y + 1] - c_ptr[y]);
}

__global__ __launch_bounds__(kBlock) void k_label_perm(const int32_t* __restrict__ rank,
                                                       int64_t n_rows, int32_t* __restrict__ perm) {
  for (int64_t y = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; y < n_rows;
       y += static_cast<int64_t>(gridDim.x) * kBlock)
    perm[label_of(rank, y)] = static_cast<int32_t>(y);
}

// A wave per 64 consecutive rows y, load-balanced over their entries (one
// contiguous range of C, read in coalesced 64-entry strips; a lane finds its
// row by a binary search over the lanes' row offsets, ds_bpermute), each entry
// written to its label's run: Q[label(y)] + its offset in the row.  Measured
// on config4 (29.4 M entries): 291 us, against 392 us for a wave per label in
// label order (gathered rows, sequential writes), 650 us for a quarter wave
// per label and 1.8-2.6 ms for the load-balanced walk in label order.
__device__ __forceinline__ uint32_t lane_u32(uint32_t v, int src) {
  return static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src << 2, static_cast<int>(v)));
}

__global__ __launch_bounds__(kBlock) void k_tile_keys(const int64_t* __restrict__ c_ptr,
                                                      const int32_t* __restrict__ c_col,
                                                      const int32_t* __restrict__ c_val,
                                                      const int32_t* __restrict__ rank,
                                                      const int64_t* __restrict__ Q,
                                                      int64_t n_rows, TileDim td, int64_t cap,
                                                      uint64_t* __restrict__ keys,
                                                      uint32_t* __restrict__ vals,
                                                      int32_t* __restrict__ status) {
  const int lane = lane_id();
  const int64_t wave0 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * (kBlock / kWave);
  for (int64_t r0 = wave0 * kWave; r0 < n_rows; r0 += nwaves * kWave) {
    const int64_t x = r0 + lane;
    const int64_t base = c_ptr[r0];
    const int64_t xe = x < n_rows ? x : n_rows;
    const uint32_t excl = static_cast<uint32_t>(c_ptr[xe] - base);
    const uint32_t total =
        static_cast<uint32_t>(c_ptr[r0 + kWave < n_rows ? r0 + kWave : n_rows] - base);
    const uint32_t labx = x < n_rows ? static_cast<uint32_t>(label_of(rank, x)) : 0u;
    // destination of strip entry i of row x: Q[label] + (i - excl), kept mod 2^32
    // (the capacity is below 2^32) relative to the strip
    const uint32_t qrel = static_cast<uint32_t>((x < n_rows ? Q[labx] : 0) - excl);
    for (uint32_t e0 = 0; e0 < total; e0 += kWave) {   // wave-uniform: every lane permutes
      const uint32_t i = e0 + static_cast<uint32_t>(lane);
      int k = 0;
#pragma unroll
      for (int step = kWave / 2; step > 0; step >>= 1)
        if (lane_u32(excl, k + step) <= i) k += step;
      const uint32_t lb = lane_u32(labx, k), qk = lane_u32(qrel, k);
      if (i < total) {
        const int64_t j = base + i;
        uint32_t c = static_cast<uint32_t>(c_val[j]);
        const uint32_t v = static_cast<uint32_t>(c_col[j]);
        if (c > 0xFFFFu) {
          if (status) *status = DPS_ERR_OVERFLOW;
          c = 0xFFFFu;
        }
        const int64_t d = static_cast<int64_t>(qk + i);
        if (d < cap) {   // past an undersized nnz_cap: k_tile_keys_pad reports the overflow
          keys[d] = (static_cast<uint64_t>(td.tile(lb)) << 32) | v;
          vals[d] = (td.local(lb) << 16) | c;
        }
      }
    }
  }
}

// Tile t's smallest denominator term, one block per tile (no atomics).
__global__ __launch_bounds__(kBlock) void k_tile_gmin(const int32_t* __restrict__ perm,
                                                      const int64_t* __restrict__ g, int64_t n_rows,
                                                      TileDim td, int64_t* __restrict__ gmin) {
  __shared__ int64_t s[kBlock];
  const int64_t lo = static_cast<int64_t>(blockIdx.x) * td.w();
  const int64_t hi = lo + td.w() < n_rows ? lo + td.w() : n_rows;
  int64_t m = INT64_MAX;
  for (int64_t lab = lo + threadIdx.x; lab < hi; lab += kBlock) {
    const int64_t v = g[perm[lab]];
    m = v < m ? v : m;
  }
  s[threadIdx.x] = m;
  __syncthreads();
  for (int o = kBlock / 2; o > 0; o >>= 1) {
    if (static_cast<int>(threadIdx.x) < o && s[threadIdx.x + o] < s[threadIdx.x])
      s[threadIdx.x] = s[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) gmin[blockIdx.x] = s[0];
}

__global__ __launch_bounds__(kBlock) void k_tile_keys_pad(const int64_t* __restrict__ c_ptr,
                                                          int64_t n_rows, int64_t cap, uint64_t pad,
                                                          uint64_t* __restrict__ keys,
                                                          uint32_t* __restrict__ vals,
                                                          int32_t* __restrict__ status) {
  const int64_t nnz = c_ptr[n_rows] - c_ptr[0];
  // the caller's nnz_cap is a host bound; C's real size is only known here
  if (nnz > cap && blockIdx.x == 0 && threadIdx.x == 0 && status) *status = DPS_ERR_OVERFLOW;
  for (int64_t i = nnz + static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < cap;
       i += static_cast<int64_t>(gridDim.x) * kBlock) {
    keys[i] = pad;
    vals[i] = 0;
  }
}

// Bucket of a sorted key, or -1 for padding.
__device__ __forceinline__ int64_t key_bucket(uint64_t key, int64_t n_mids, int64_t T) {
  const int64_t v = static_cast<int64_t>(key & 0xFFFFFFFFu);
  return v >= n_mids ? -1 : v * T + static_cast<int64_t>(key >> 32);
}

// Per sorted pair: its pieces (0 past nnz), the first / one-past-last index of
// its bucket's run (bstart / bend), and the bucket maximum (C > 1 only:
// k_round4 style, the counts pass raises a non-empty bucket's maximum to 1) as
// a segmented max over the wave's lanes -- one atomic per bucket and wave.
__global__ __launch_bounds__(kBlock) void k_sorted_runs(const uint64_t* __restrict__ keys,
                                                        const uint32_t* __restrict__ vals,
                                                        int64_t cap, int64_t n_mids, int64_t T,
                                                        int fmt, uint32_t* __restrict__ pieces,
                                                        uint32_t* __restrict__ bstart,
                                                        uint32_t* __restrict__ bend,
                                                        uint32_t* __restrict__ maxc) {
  const int lane = lane_id();
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t w0 = static_cast<int64_t>(blockIdx.x) * kBlock + (threadIdx.x & ~(kWave - 1));
       w0 < cap; w0 += stride) {
    const int64_t i = w0 + lane;
    const bool valid = i < cap;
    const uint64_t key = valid ? keys[i] : ~0ull;
    const int64_t b = valid ? key_bucket(key, n_mids, T) : -1;
    uint32_t m = 0;
    if (b >= 0) {
      const uint32_t v = vals[i];
      const uint32_t c = v & 0xFFFFu, l = v >> 16;
      pieces[i] = n_pieces(fmt, c, l);
      m = c;
      if (i == 0 || keys[i - 1] != key) bstart[b] = static_cast<uint32_t>(i);
      if (i + 1 == cap || keys[i + 1] != key) bend[b] = static_cast<uint32_t>(i + 1);
    } else if (valid) {
      pieces[i] = 0;
    }
    if (!maxc) continue;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const uint32_t mo = __shfl_up(m, o, kWave);
      const uint64_t ko = __shfl_up(key, o, kWave);
      if (lane >= o && ko == key) m = m > mo ? m : mo;
    }
    const uint64_t kn = __shfl_down(key, 1, kWave);
    const bool last = lane == kWave - 1 || kn != key;
    if (b >= 0 && last && m > 1) atomicMax(&maxc[b], m);
  }
}

// Bucket b's padded count (cnt[], scanned into the layout).
__global__ __launch_bounds__(kBlock) void k_sorted_counts(const uint32_t* __restrict__ bstart,
                                                          const uint32_t* __restrict__ bend,
                                                          const int64_t* __restrict__ P, int64_t nb,
                                                          uint32_t per16, uint32_t* __restrict__ cnt,
                                                          uint32_t* __restrict__ maxc) {
  for (int64_t b = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; b < nb;
       b += static_cast<int64_t>(gridDim.x) * kBlock) {
    const uint32_t s0 = bstart[b], s1 = bend[b];
    const uint32_t n = s1 > s0 ? static_cast<uint32_t>(P[s1] - P[s0]) : 0u;
    cnt[b] = padded_count(n, per16);
    if (maxc && n > 0 && maxc[b] == 0) maxc[b] = 1;
  }
}

// Each pair's entries at its bucket's offset + the pieces before it in the
// run; the run's last pair also writes the bucket's padding.
__global__ __launch_bounds__(kBlock) void k_sorted_write(const uint64_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ vals,
                                                         int64_t cap, int64_t n_mids, int64_t T,
                                                         int fmt, uint32_t lab_mask,
                                                         const int64_t* __restrict__ P,
                                                         const uint32_t* __restrict__ bstart,
                                                         const int64_t* __restrict__ off,
                                                         uint32_t* __restrict__ ent) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < cap;
       i += static_cast<int64_t>(gridDim.x) * kBlock) {
    const uint64_t key = keys[i];
    const int64_t b = key_bucket(key, n_mids, T);
    if (b < 0) continue;
    const uint32_t v = vals[i];
    const int64_t p0 = P[bstart[b]];
    put_entry(fmt, ent, off[b] + (P[i] - p0), v & 0xFFFFu, v >> 16);
    if (i + 1 == cap || keys[i + 1] != key) {
      const int64_t i0 = off[b] + (P[i + 1] - p0);
      pad_bucket(i0, off[b + 1] - i0, lab_mask, fmt, ent);
    }
  }
}

}  // namespace
}  // namespace dps

using namespace dps;


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

int64_t dps_ct_tiles_ent_capacity(int64_t nnz, int64_t sum_c, int64_t n_mids,
                                  int64_t n_targets, int32_t tile_w) {
  if (tile_w <= 0 || nnz < 0 || sum_c < nnz) return 0;
  const int64_t T = (n_targets + tile_w - 1) / tile_w;
  const int64_t nb = n_mids * (T > 0 ? T : 1);
  if (tile_fmt(tile_dim(tile_w).shift) == kFmt32) return nnz + 3 * (nb < nnz ? nb : nnz) + 4;
  // 16-bit entries: power-of-two pieces, at most (c + 1) / 2 <= 1 + (c - 1) / 2
  // per C entry; up to 9 padding entries per non-empty bucket; two entries per
  // uint32 word
  const int64_t pieces = nnz + (sum_c - nnz + 1) / 2;
  return (pieces + 9 * (nb < pieces ? nb : pieces) + 1) / 2 + 4;
}

size_t dps_ct_tiles_workspace_size(int64_t n_mids, int64_t n_targets, int32_t tile_w) {
  if (tile_w <= 0) return 0;
  const int64_t T = (n_targets + tile_w - 1) / tile_w;
  const int64_t nb = n_mids * (T > 0 ? T : 1);
  const int64_t np = nb * tile_parts(n_mids, tile_w);   // part slots (blk path) or buckets
  size_t s = 0;
  s += align_up(static_cast<size_t>(nb + 1) * sizeof(uint32_t));  // cnt
  s += align_up(static_cast<size_t>(nb + 1) * sizeof(uint32_t));  // cursor
  s += align_up(static_cast<size_t>(np + 1) * sizeof(int64_t));   // off64 (per part)
  s += align_up(scan_workspace_size(np + 1));
  s += align_up(static_cast<size_t>(np + 1) * sizeof(uint32_t));  // cntp
  s += align_up(static_cast<size_t>(np + 1) * sizeof(uint32_t));  // mxp
  s += align_up(static_cast<size_t>(np + 1) * sizeof(uint32_t));  // curp
  s += align_up(static_cast<size_t>(np + 1) * sizeof(uint32_t));  // part_n
  s += align_up(static_cast<size_t>(n_targets > 0 ? n_targets : 1) * sizeof(int32_t));  // perm
  return s + 1024;
}

int dps_ct_tiles_sums(const uint32_t* tile_off, const uint32_t* tile_ent, int64_t n_buckets,
                      int32_t tile_w, uint32_t* tile_sum, void* stream) {
  DPS_REQUIRE(n_buckets >= 0, DPS_ERR_INVALID, "bad n_buckets");
  const TileDim td = tile_dim(tile_w);
  DPS_REQUIRE(td.shift >= 0, DPS_ERR_INVALID,
              "tile_w must be a power of two in [256, 65536], 7680 or 15360");
  if (n_buckets == 0) return DPS_OK;
  DPS_REQUIRE(tile_off && tile_ent && tile_sum, DPS_ERR_INVALID, "null array");
  const int fmt = tile_fmt(td.shift);
  k_tile_sums<<<grid_for(n_buckets * 16, kBlock), kBlock, 0, static_cast<hipStream_t>(stream)>>>(
      tile_off, tile_ent, n_buckets, fmt, tile_sum);
  DPS_LAUNCHED();
  return DPS_OK;
}

int dps_ct_tiles_build(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                       const int64_t* g, const int32_t* t_rank, int64_t n_targets, int64_t n_mids,
                       int32_t tile_w, uint32_t* tile_off, uint32_t* tile_ent, uint32_t* tile_maxc,
                       int64_t* tile_gmin, int32_t* status_dev, void* ws, size_t ws_bytes,
                       void* stream) {
  const TileDim td = tile_dim(tile_w);
  const int shift = td.shift;
  DPS_REQUIRE(shift >= 8 && shift <= 16, DPS_ERR_UNSUPPORTED,
              "tile_w must be a power of two in [256, 65536], 7680 or 15360, got %d", tile_w);
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
  // block-local LDS counting, parts per tile, one block per kBlkMids mids
  const bool blk = !tile_global(n_mids);
  const int n_ranges = static_cast<int>(n_mids > 0 ? (n_mids + kBlkMids - 1) / kBlkMids : 1);
  const int P = static_cast<int>(tile_parts(n_mids, tile_w));
  const int64_t np = nb * P;
  Carve c(ws, ws_bytes);
  uint32_t* cnt = c.take<uint32_t>(nb + 1);
  uint32_t* cursor = c.take<uint32_t>(nb + 1);
  int64_t* off64 = c.take<int64_t>(np + 1);
  const size_t scan_ws = scan_workspace_size(np + 1);
  void* sws = c.take<char>(scan_ws);
  uint32_t* cntp = c.take<uint32_t>(np + 1);
  uint32_t* mxp = c.take<uint32_t>(np + 1);
  uint32_t* curp = c.take<uint32_t>(np + 1);
  uint32_t* part_n = c.take<uint32_t>(np + 1);   // entries per part (nblk <= np)
  int32_t* perm = c.take<int32_t>(n_targets > 0 ? n_targets : 1);
  DPS_REQUIRE(c.ok, DPS_ERR_WORKSPACE, "tiles workspace carve failed");
  const int lpb = tile_lpb(tile_w);
  const int64_t nblk = (n_targets + lpb - 1) / lpb;
  const int S = tile_sub();
  DPS_REQUIRE(nblk * S * n_ranges < INT32_MAX, DPS_ERR_OVERFLOW, "too many tile-build blocks");
  const int fmt = tile_fmt(shift);
  const bool p16 = fmt != kFmt32;   // 16-bit entries: counts and offsets are in entries
  const uint32_t per16 = p16 ? 8u : 4u;
  const bool fused_parts = blk && n_targets > 0 && nblk <= kPartLds;
  if (blk) {   // every counter, the status word and the tile minima in one launch
    FillSet fs;
    fs.add(part_n, nblk + 1, 0u);
    fs.add(cntp, np + 1, 0u);
    fs.add(mxp, np + 1, 0u);
    fs.add(curp, np + 1, 0u);
    if (status_dev) fs.add(status_dev, 1, 0u);
    if (tile_gmin && T > 0) fs.add(tile_gmin, 2 * T, 0x7F7F7F7Fu);
    if (tile_maxc) fs.add(tile_maxc + nb, 1, 0u);
    DPS_HIP_RET(fill_set(fs, st));
  }
  if (fused_parts) {
    k_invert_and_parts<<<grid_for(n_targets, kBlock, 1024), kBlock, 0, st>>>(
        t_rank, c_ptr, n_targets, lpb, static_cast<int>(nblk), perm, part_n);
    DPS_LAUNCHED();
  } else if (blk && t_rank && n_targets > 0) {
    k_tile_invert<<<grid_for(n_targets, kBlock), kBlock, 0, st>>>(t_rank, n_targets, perm);
    DPS_LAUNCHED();
  }
  const int32_t* perm_or_null = t_rank ? perm : nullptr;
  if (!blk) {
    if (status_dev) DPS_HIP_RET(hipMemsetAsync(status_dev, 0, sizeof(int32_t), st));
    if (tile_gmin && T > 0) DPS_HIP_RET(hipMemsetAsync(tile_gmin, 0x7F, T * sizeof(int64_t), st));
  }
  if (blk) {
    if (!fused_parts) {
      if (n_targets > 0) {
        k_part_entries<<<grid_for(n_targets, kBlock), kBlock, 0, st>>>(c_ptr, perm_or_null,
                                                                       n_targets, lpb, part_n);
        DPS_LAUNCHED();
      }
    }
    if (n_targets > 0 && nb > 0) {
      k_tile_count_blk<<<static_cast<unsigned>(nblk * S * n_ranges), kBlkThreads, 0, st>>>(
          c_ptr, c_col, c_val, perm_or_null, tile_gmin ? g : nullptr, n_targets, n_mids, td, T,
          lpb, P, S, n_ranges, part_n, cntp, mxp,
          reinterpret_cast<unsigned long long*>(tile_gmin), status_dev);
      DPS_LAUNCHED();
    }
    if (nb > 0) {
      k_tile_parts_fix<<<grid_for(nb, kBlock), kBlock, 0, st>>>(cntp, mxp, nb, P, per16, cnt,
                                                                 tile_maxc);
      DPS_LAUNCHED();
    }
    DPS_HIP_RET(scan_exclusive<uint32_t>(cntp, off64, np, sws, scan_ws, st));
    k_tile_off32<<<grid_for(nb + 1, kBlock), kBlock, 0, st>>>(off64, P, nb, p16 ? 1 : 0, tile_off);
    DPS_LAUNCHED();
    if (n_targets > 0 && nb > 0) {
      k_tile_scatter_blk<<<static_cast<unsigned>(nblk * S * n_ranges), kBlkThreads, 0, st>>>(
          c_ptr, c_col, c_val, perm_or_null, n_targets, n_mids, td, T, lpb, P, S, n_ranges,
          part_n, off64, curp, tile_ent);
      DPS_LAUNCHED();
    }
    if (nb > 0) {
      k_tile_pad<<<grid_for(nb, kBlock), kBlock, 0, st>>>(off64, P, cnt, nb, pad_mask(td), fmt,
                                                          tile_ent);
      DPS_LAUNCHED();
    }
    return bank_order(p16, nb, tile_off, tile_ent, st);
  }
  // many mids: global-atomic counting sort into (v, t) buckets
  DPS_HIP_RET(hipMemsetAsync(cnt, 0, (nb + 1) * sizeof(uint32_t), st));
  DPS_HIP_RET(hipMemsetAsync(cursor, 0, (nb + 1) * sizeof(uint32_t), st));
  if (tile_maxc) DPS_HIP_RET(hipMemsetAsync(tile_maxc, 0, (nb + 1) * sizeof(uint32_t), st));
  if (n_targets > 0 && nb > 0) {
    k_tile_count<<<grid_for(n_targets * kWave, kBlock, 2048), kBlock, 0, st>>>(
        c_ptr, c_col, c_val, t_rank, g, n_targets, td, T, cnt, tile_maxc,
        reinterpret_cast<unsigned long long*>(tile_gmin), status_dev);
    DPS_LAUNCHED();
  }
  if (nb > 0) {
    k_round4<<<grid_for(nb, kBlock), kBlock, 0, st>>>(cnt, nb, per16, tile_maxc);
    DPS_LAUNCHED();
  }
  DPS_HIP_RET(scan_exclusive<uint32_t>(cnt, off64, nb, sws, scan_ws, st));
  k_tile_off32<<<grid_for(nb + 1, kBlock), kBlock, 0, st>>>(off64, 1, nb, p16 ? 1 : 0, tile_off);
  DPS_LAUNCHED();
  if (n_targets > 0 && nb > 0) {
    k_tile_scatter<<<grid_for(n_targets * kWave, kBlock), kBlock, 0, st>>>(
        c_ptr, c_col, c_val, t_rank, n_targets, td, T, off64, cursor, tile_ent);
    DPS_LAUNCHED();
  }
  if (nb > 0) {
    k_tile_pad<<<grid_for(nb, kBlock), kBlock, 0, st>>>(off64, 1, cursor, nb, pad_mask(td), fmt,
                                                        tile_ent);
    DPS_LAUNCHED();
  }
  return bank_order(p16, nb, tile_off, tile_ent, st);
}

size_t dps_ct_tiles_workspace_size2(int64_t n_mids, int64_t n_targets, int32_t tile_w,
                                    int64_t nnz_cap) {
  const size_t base = dps_ct_tiles_workspace_size(n_mids, n_targets, tile_w);
  if (tile_w <= 0 || !tile_global(n_mids)) return base;
  const int64_t T = (n_targets + tile_w - 1) / tile_w;
  const size_t nb = static_cast<size_t>(n_mids * (T > 0 ? T : 1));
  const size_t cap = static_cast<size_t>(nnz_cap > 0 ? nnz_cap : 1);
  size_t s = 0;
  s += 2 * align_up(cap * sizeof(uint64_t));          // keys, sorted keys
  s += 2 * align_up(cap * sizeof(uint32_t));          // vals, sorted vals
  s += align_up(cap * sizeof(uint32_t));              // pieces
  s += align_up((cap + 1) * sizeof(int64_t));         // P
  s += align_up(scan_workspace_size(static_cast<int64_t>(cap)));
  s += 2 * align_up((nb + 1) * sizeof(uint32_t));     // bstart, bend
  s += align_up(radix_sort_workspace_size(static_cast<int64_t>(cap)));
  const size_t nt = static_cast<size_t>(n_targets > 0 ? n_targets : 1);
  s += align_up((nt + 1) * sizeof(uint32_t)) + align_up((nt + 1) * sizeof(int64_t));  // len, Q
  s += align_up(nt * sizeof(int32_t));                                                // perm
  s += align_up(scan_workspace_size(static_cast<int64_t>(nt)));
  return base + s + 1024;
}

int dps_ct_tiles_build2(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                        const int64_t* g, const int32_t* t_rank, int64_t n_targets, int64_t n_mids,
                        int32_t tile_w, int64_t nnz_cap, uint32_t* tile_off, uint32_t* tile_ent,
                        uint32_t* tile_maxc, int64_t* tile_gmin, int32_t* status_dev, void* ws,
                        size_t ws_bytes, void* stream) {
  if (!tile_global(n_mids))
    return dps_ct_tiles_build(c_ptr, c_col, c_val, g, t_rank, n_targets, n_mids, tile_w, tile_off,
                              tile_ent, tile_maxc, tile_gmin, status_dev, ws, ws_bytes, stream);
  const TileDim td = tile_dim(tile_w);
  const int shift = td.shift;
  DPS_REQUIRE(shift >= 8 && shift <= 16, DPS_ERR_UNSUPPORTED,
              "tile_w must be a power of two in [256, 65536], 7680 or 15360, got %d", tile_w);
  DPS_REQUIRE(n_targets >= 0 && n_mids >= 0 && nnz_cap >= 0, DPS_ERR_INVALID, "negative size");
  DPS_REQUIRE(n_targets < INT32_MAX && nnz_cap < UINT32_MAX, DPS_ERR_OVERFLOW,
              "n_targets / nnz capacity exceed 32 bits");
  DPS_REQUIRE(!tile_gmin || g, DPS_ERR_INVALID, "tile_gmin needs g");
  DPS_REQUIRE(reinterpret_cast<uintptr_t>(ws) % 256 == 0, DPS_ERR_WORKSPACE,
              "workspace not 256-byte aligned");
  DPS_REQUIRE(ws_bytes >= dps_ct_tiles_workspace_size2(n_mids, n_targets, tile_w, nnz_cap),
              DPS_ERR_WORKSPACE, "tiles workspace too small");
  auto st = static_cast<hipStream_t>(stream);
  const int64_t T = (n_targets + tile_w - 1) / tile_w;
  const int64_t nb = n_mids * T;
  const int64_t cap = nnz_cap > 0 ? nnz_cap : 1;
  Carve c(ws, ws_bytes);
  uint32_t* cnt = c.take<uint32_t>(nb + 1);
  int64_t* off64 = c.take<int64_t>(nb + 1);
  const size_t scan_b = scan_workspace_size(nb + 1);
  void* sws_b = c.take<char>(scan_b);
  uint64_t* keys = c.take<uint64_t>(cap);
  uint64_t* keys_s = c.take<uint64_t>(cap);
  uint32_t* vals = c.take<uint32_t>(cap);
  uint32_t* vals_s = c.take<uint32_t>(cap);
  uint32_t* pieces = c.take<uint32_t>(cap);
  int64_t* P = c.take<int64_t>(cap + 1);
  const size_t scan_e = scan_workspace_size(cap);
  void* sws_e = c.take<char>(scan_e);
  uint32_t* bstart = c.take<uint32_t>(nb + 1);
  uint32_t* bend = c.take<uint32_t>(nb + 1);
  const size_t rs_bytes = radix_sort_workspace_size(cap);
  void* rws = c.take<char>(rs_bytes);
  const int64_t nt = n_targets > 0 ? n_targets : 1;
  uint32_t* len = c.take<uint32_t>(nt + 1);
  int64_t* Q = c.take<int64_t>(nt + 1);
  int32_t* perm = c.take<int32_t>(nt);
  const size_t scan_q = scan_workspace_size(nt);
  void* sws_q = c.take<char>(scan_q);
  DPS_REQUIRE(c.ok, DPS_ERR_WORKSPACE, "tiles workspace carve failed");
  const int fmt = tile_fmt(shift);
  const uint32_t per16 = fmt != kFmt32 ? 8u : 4u;
  {
    FillSet fs;
    fs.add(bstart, nb + 1, 0u);
    fs.add(bend, nb + 1, 0u);
    if (status_dev) fs.add(status_dev, 1, 0u);
    if (tile_gmin && T > 0) fs.add(tile_gmin, 2 * T, 0x7F7F7F7Fu);
    if (tile_maxc) fs.add(tile_maxc, nb + 1, 0u);
    DPS_HIP_RET(fill_set(fs, st));
  }
  if (n_targets > 0) {
    k_label_len<<<grid_for(n_targets, kBlock), kBlock, 0, st>>>(c_ptr, t_rank, n_targets, len);
    DPS_LAUNCHED();
    k_label_perm<<<grid_for(n_targets, kBlock), kBlock, 0, st>>>(t_rank, n_targets, perm);
    DPS_LAUNCHED();
    DPS_HIP_RET(scan_exclusive<uint32_t>(len, Q, n_targets, sws_q, scan_q, st));
    k_tile_keys<<<grid_for((n_targets + kWave - 1) / kWave * kWave, kBlock, 4096), kBlock, 0, st>>>(
        c_ptr, c_col, c_val, t_rank, Q, n_targets, td, cap, keys, vals, status_dev);
    DPS_LAUNCHED();
    if (tile_gmin) {
      k_tile_gmin<<<static_cast<unsigned>(T), kBlock, 0, st>>>(perm, g, n_targets, td, tile_gmin);
      DPS_LAUNCHED();
    }
  }
  k_tile_keys_pad<<<grid_for(cap, kBlock), kBlock, 0, st>>>(c_ptr, n_targets, cap,
                                                           static_cast<uint64_t>(n_mids), keys, vals,
                                                           status_dev);
  DPS_LAUNCHED();
  int key_bits = 1;
  while ((int64_t(1) << key_bits) <= n_mids) ++key_bits;   // n_mids itself is the pad mid
  DPS_HIP_RET(radix_sort_pairs(keys, vals, keys_s, vals_s, cap, key_bits, rws, rs_bytes, st));
  k_sorted_runs<<<grid_for(cap, kBlock), kBlock, 0, st>>>(keys_s, vals_s, cap, n_mids, T, fmt,
                                                         pieces, bstart, bend, tile_maxc);
  DPS_LAUNCHED();
  DPS_HIP_RET(scan_exclusive<uint32_t>(pieces, P, cap, sws_e, scan_e, st));
  if (nb > 0) {
    k_sorted_counts<<<grid_for(nb, kBlock), kBlock, 0, st>>>(bstart, bend, P, nb, per16, cnt,
                                                            tile_maxc);
    DPS_LAUNCHED();
  }
  DPS_HIP_RET(scan_exclusive<uint32_t>(cnt, off64, nb, sws_b, scan_b, st));
  k_tile_off32<<<grid_for(nb + 1, kBlock), kBlock, 0, st>>>(off64, 1, nb, fmt != kFmt32 ? 1 : 0,
                                                           tile_off);
  DPS_LAUNCHED();
  k_sorted_write<<<grid_for(cap, kBlock), kBlock, 0, st>>>(keys_s, vals_s, cap, n_mids, T, fmt,
                                                          pad_mask(td), P,
                                                          bstart, off64, tile_ent);
  DPS_LAUNCHED();
  return bank_order(fmt != kFmt32, nb, tile_off, tile_ent, st);
}

size_t dps_ct_tiles_workspace_size_dual(int64_t n_mids, int64_t n_targets, int32_t tile_w,
                                        int64_t nnz_cap) {
  const TileDim tdA = tile_dim(tile_w);
  if (tdA.shift != 14 || tile_w <= 0) return 0;
  const int32_t hw = tile_w / 2;
  const size_t a2 = dps_ct_tiles_workspace_size2(n_mids, n_targets, tile_w, nnz_cap);
  const size_t b2 = dps_ct_tiles_workspace_size2(n_mids, n_targets, hw, nnz_cap);
  const size_t fb = a2 > b2 ? a2 : b2;                 // the two-call path
  if (tile_global(n_mids)) return fb;
  const int64_t TA = (n_targets + tile_w - 1) / tile_w, TB = (n_targets + hw - 1) / hw;
  const int64_t nbA = n_mids * (TA > 0 ? TA : 1), nbB = n_mids * (TB > 0 ? TB : 1);
  const int lpb = tile_lpb(tile_w);
  const int64_t npA = nbA * (tile_w / lpb), npB = nbB * (hw / lpb);
  const int64_t nblk = (n_targets + lpb - 1) / lpb;
  size_t s = 0;
  s += align_up(static_cast<size_t>(nbA + 1) * 4) + align_up(static_cast<size_t>(nbB + 1) * 4);
  s += align_up(static_cast<size_t>(npA + 1) * 8) + align_up(static_cast<size_t>(npB + 1) * 8);
  s += align_up(scan_workspace_size((npA > npB ? npA : npB) + 1));
  s += 3 * align_up(static_cast<size_t>(npA + 1) * 4) + 3 * align_up(static_cast<size_t>(npB + 1) * 4);
  s += align_up(static_cast<size_t>(nblk + 1) * 4);
  s += align_up(static_cast<size_t>(n_targets > 0 ? n_targets : 1) * 4);
  s += 1024;
  return s > fb ? s : fb;
}

int dps_ct_tiles_build_dual(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                            const int64_t* g, const int32_t* t_rank, int64_t n_targets,
                            int64_t n_mids, int32_t tile_w, int64_t nnz_cap, uint32_t* tile_off,
                            uint32_t* tile_ent, int64_t tile_ent_words, uint32_t* tile_maxc,
                            int64_t* tile_gmin, uint32_t* half_off, uint32_t* half_ent,
                            int64_t half_ent_words, uint32_t* half_maxc, int32_t* status_dev,
                            int32_t* half_status, const int32_t* hv_slot, int32_t n_hv,
                            uint16_t* hv_c, void* ws, size_t ws_bytes, void* stream) {
  const TileDim tdA = tile_dim(tile_w), tdB = tile_dim(tile_w / 2);
  DPS_REQUIRE(tdA.shift == 14 && tdB.shift == 13 && tdA.t15 == tdB.t15, DPS_ERR_UNSUPPORTED,
              "the dual build takes tile_w 16384 or 15360 (4-bit tiles), got %d", tile_w);
  DPS_REQUIRE(n_targets >= 0 && n_mids >= 0 && nnz_cap >= 0, DPS_ERR_INVALID, "negative size");
  DPS_REQUIRE(n_targets < INT32_MAX, DPS_ERR_OVERFLOW, "n_targets exceeds int32");
  DPS_REQUIRE(!tile_gmin || g, DPS_ERR_INVALID, "tile_gmin needs g");
  DPS_REQUIRE(tile_off && tile_ent && half_off && half_ent, DPS_ERR_INVALID, "null tile arrays");
  DPS_REQUIRE(!hv_c || (hv_slot && n_hv >= 1 && n_hv <= 64), DPS_ERR_INVALID,
              "hv_c needs hv_slot and n_hv in [1, 64]");
  DPS_REQUIRE(reinterpret_cast<uintptr_t>(ws) % 256 == 0, DPS_ERR_WORKSPACE,
              "workspace not 256-byte aligned");
  DPS_REQUIRE(ws_bytes >= dps_ct_tiles_workspace_size_dual(n_mids, n_targets, tile_w, nnz_cap),
              DPS_ERR_WORKSPACE, "tiles workspace too small");
  const int32_t hw = tile_w / 2;
  // the heavy table from the count walk: zeroed with the counters (as words:
  // even n_hv and a 4-byte aligned table), else by dps_heavy_table after
  const bool hv_fused = hv_c && (n_hv & 1) == 0 && (reinterpret_cast<uintptr_t>(hv_c) & 3u) == 0;
  // many mids, or 16-bit entry offsets beyond the scatter's 32-bit cursors:
  // the two builds one after the other (they reuse the workspace)
  if (tile_global(n_mids) || 2 * tile_ent_words >= (int64_t(1) << 32) ||
      2 * half_ent_words >= (int64_t(1) << 32)) {
    int rc = dps_ct_tiles_build2(c_ptr, c_col, c_val, g, t_rank, n_targets, n_mids, tile_w,
                                 nnz_cap, tile_off, tile_ent, tile_maxc, tile_gmin,
                                 status_dev, ws, ws_bytes, stream);
    if (rc != DPS_OK) return rc;
    rc = dps_ct_tiles_build2(c_ptr, c_col, c_val, nullptr, t_rank, n_targets, n_mids, hw,
                             nnz_cap, half_off, half_ent, half_maxc, nullptr, half_status, ws,
                             ws_bytes, stream);
    if (rc != DPS_OK || !hv_c) return rc;
    return dps_heavy_table(c_ptr, c_col, c_val, t_rank, n_targets, hv_slot, n_hv, hv_c, stream);
  }
  auto st = static_cast<hipStream_t>(stream);
  const int64_t TA = (n_targets + tile_w - 1) / tile_w, TB = (n_targets + hw - 1) / hw;
  const int64_t nbA = n_mids * TA, nbB = n_mids * TB;
  const int n_ranges = static_cast<int>(n_mids > 0 ? (n_mids + kBlkMids - 1) / kBlkMids : 1);
  const int lpb = tile_lpb(tile_w);
  const int PA = tile_w / lpb, PB = hw / lpb;
  const int64_t npA = nbA * PA, npB = nbB * PB;
  const int64_t nblk = (n_targets + lpb - 1) / lpb;
  const int S = tile_sub();
  DPS_REQUIRE(nblk * S * n_ranges < INT32_MAX, DPS_ERR_OVERFLOW, "too many tile-build blocks");
  Carve c(ws, ws_bytes);
  uint32_t* cntA = c.take<uint32_t>(nbA + 1);
  uint32_t* cntB = c.take<uint32_t>(nbB + 1);
  int64_t* offA = c.take<int64_t>(npA + 1);
  int64_t* offB = c.take<int64_t>(npB + 1);
  const size_t scan_ws = scan_workspace_size((npA > npB ? npA : npB) + 1);
  void* sws = c.take<char>(scan_ws);
  uint32_t* cntpA = c.take<uint32_t>(npA + 1);
  uint32_t* mxpA = c.take<uint32_t>(npA + 1);
  uint32_t* curpA = c.take<uint32_t>(npA + 1);
  uint32_t* cntpB = c.take<uint32_t>(npB + 1);
  uint32_t* mxpB = c.take<uint32_t>(npB + 1);
  uint32_t* curpB = c.take<uint32_t>(npB + 1);
  uint32_t* part_n = c.take<uint32_t>(nblk + 1);
  int32_t* perm = c.take<int32_t>(n_targets > 0 ? n_targets : 1);
  DPS_REQUIRE(c.ok, DPS_ERR_WORKSPACE, "tiles workspace carve failed");
  {
    FillSet fs;   // every counter, both status words and the tile minima in one launch
    fs.add(part_n, nblk + 1, 0u);
    fs.add(cntpA, npA + 1, 0u);
    fs.add(mxpA, npA + 1, 0u);
    fs.add(curpA, npA + 1, 0u);
    fs.add(cntpB, npB + 1, 0u);
    fs.add(mxpB, npB + 1, 0u);
    fs.add(curpB, npB + 1, 0u);
    if (status_dev) fs.add(status_dev, 1, 0u);
    if (half_status) fs.add(half_status, 1, 0u);
    if (tile_gmin && TA > 0) fs.add(tile_gmin, 2 * TA, 0x7F7F7F7Fu);
    if (tile_maxc) fs.add(tile_maxc + nbA, 1, 0u);
    if (half_maxc) fs.add(half_maxc + nbB, 1, 0u);
    if (hv_fused && n_targets > 0)
      fs.add(reinterpret_cast<uint32_t*>(hv_c), n_targets * n_hv / 2, 0u);
    DPS_HIP_RET(fill_set(fs, st));
  }
  if (n_targets > 0 && nblk <= kPartLds) {
    k_invert_and_parts<<<grid_for(n_targets, kBlock, 1024), kBlock, 0, st>>>(
        t_rank, c_ptr, n_targets, lpb, static_cast<int>(nblk), perm, part_n);
    DPS_LAUNCHED();
  } else if (n_targets > 0) {
    if (t_rank) {
      k_tile_invert<<<grid_for(n_targets, kBlock), kBlock, 0, st>>>(t_rank, n_targets, perm);
      DPS_LAUNCHED();
    }
    k_part_entries<<<grid_for(n_targets, kBlock), kBlock, 0, st>>>(c_ptr, t_rank ? perm : nullptr,
                                                                   n_targets, lpb, part_n);
    DPS_LAUNCHED();
  }
  const int32_t* perm_or_null = t_rank ? perm : nullptr;
  const int fmtA = tile_fmt(tdA.shift), fmtB = tile_fmt(tdB.shift);
  const unsigned grid = static_cast<unsigned>(nblk * S * n_ranges);
  if (n_targets > 0 && nbA > 0) {
    k_tile_count_dual<<<grid, kBlkThreads, 0, st>>>(
        c_ptr, c_col, c_val, perm_or_null, tile_gmin ? g : nullptr, n_targets, n_mids, tdA, TA, tdB,
        TB, lpb, PA, PB, S, n_ranges, part_n, cntpA, mxpA, cntpB, mxpB,
        reinterpret_cast<unsigned long long*>(tile_gmin), status_dev, hv_slot, n_hv,
        hv_fused ? hv_c : nullptr);
    DPS_LAUNCHED();
  }
  if (hv_c && !hv_fused) {
    const int rc = dps_heavy_table(c_ptr, c_col, c_val, t_rank, n_targets, hv_slot, n_hv, hv_c, stream);
    if (rc != DPS_OK) return rc;
  }
  if (nbA > 0) {
    k_tile_parts_fix<<<grid_for(nbA, kBlock), kBlock, 0, st>>>(cntpA, mxpA, nbA, PA, 8u, cntA,
                                                                tile_maxc);
    DPS_LAUNCHED();
    k_tile_parts_fix<<<grid_for(nbB, kBlock), kBlock, 0, st>>>(cntpB, mxpB, nbB, PB, 8u, cntB,
                                                                half_maxc);
    DPS_LAUNCHED();
  }
  DPS_HIP_RET(scan_exclusive<uint32_t>(cntpA, offA, npA, sws, scan_ws, st));
  k_tile_off32<<<grid_for(nbA + 1, kBlock), kBlock, 0, st>>>(offA, PA, nbA, 1, tile_off);
  DPS_LAUNCHED();
  DPS_HIP_RET(scan_exclusive<uint32_t>(cntpB, offB, npB, sws, scan_ws, st));
  k_tile_off32<<<grid_for(nbB + 1, kBlock), kBlock, 0, st>>>(offB, PB, nbB, 1, half_off);
  DPS_LAUNCHED();
  if (n_targets > 0 && nbA > 0) {
    k_tile_scatter_dual<<<grid, kBlkThreads, 0, st>>>(
        c_ptr, c_col, c_val, perm_or_null, n_targets, n_mids, tdA, TA, tdB, TB, lpb, PA, PB, S,
        n_ranges, part_n, offA, curpA, tile_ent, offB, curpB, half_ent);
    DPS_LAUNCHED();
  }
  if (nbA > 0) {
    k_tile_pad<<<grid_for(nbA, kBlock), kBlock, 0, st>>>(offA, PA, cntA, nbA, pad_mask(tdA), fmtA,
                                                         tile_ent);
    DPS_LAUNCHED();
    k_tile_pad<<<grid_for(nbB, kBlock), kBlock, 0, st>>>(offB, PB, cntB, nbB, pad_mask(tdB), fmtB,
                                                         half_ent);
    DPS_LAUNCHED();
  }
  const int rc = bank_order(true, nbA, tile_off, tile_ent, st);
  if (rc != DPS_OK) return rc;
  return bank_order(true, nbB, half_off, half_ent, st);
}

int dps_walk_row(const int32_t* src_col, const int32_t* src_val, int64_t src_len,
                 const int32_t* t_perm, int64_t n_targets, int64_t n_mids, int32_t tile_w,
                 const uint32_t* tile_off, const uint32_t* tile_ent, int64_t* out_m,
                 void* stream) {
  (void)n_mids;
  const TileDim td = tile_dim(tile_w);
  DPS_REQUIRE(td.shift >= 8 && td.shift <= 16, DPS_ERR_UNSUPPORTED, "bad tile_w %d", tile_w);
  DPS_REQUIRE(src_len >= 0 && n_targets >= 0, DPS_ERR_INVALID, "negative size");
  auto st = static_cast<hipStream_t>(stream);
  const int64_t T = (n_targets + tile_w - 1) / tile_w;
  if (T == 0) return DPS_OK;
  DPS_HIP_RET(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_walk_row),
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  static_cast<int>((tile_w < 32768 ? tile_w : 32768) *
                                                   sizeof(int32_t))));
  k_walk_row<<<static_cast<unsigned>(T), kBlock,
               static_cast<size_t>(tile_w < 32768 ? tile_w : 32768) * sizeof(int32_t),
               st>>>(src_col, src_val, src_len, n_targets, td, T, tile_off, tile_ent, t_perm,
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
