// Device helpers shared by the hot-path kernels (dps_cct.hip: general kernel,
// dps_cct1.hip: lean one-wave kernel for W = 8192).  See dps_cct.hip's header
// for the operands and the algorithm.
#pragma once

#include "dps_common.hpp"

namespace dps {

// Kernel parameters (shared by both kernels; the lean kernel ignores the
// multi-wave fields).
struct CctParams {
  const int64_t* c_ptr;
  const int32_t* c_col;
  const int32_t* c_val;
  const int64_t* g;          // original order (sources)
  const int64_t* g_t;        // label order (targets, ascending)
  const int32_t* t_perm;     // label -> original (nullable = identity)
  const int32_t* t_rank;     // original -> label (nullable = identity)
  const uint32_t* tile_off;
  const uint32_t* tile_ent;
  const uint32_t* tile_maxc; // tile_off stands in when no bounds are given
  bool use_bounds;           // false: no skipping, every tile wide
  const int64_t* tile_gmin;
  int64_t n_targets;
  int64_t T;
  int shift;                 // the entry format: 13 u8, 14 4-bit, 15-16 32-bit entries
  int tile_w;                // targets per tile: 2^shift, or 15 * 2^(shift - 4) (the T15
                             // layout of dps_cct1.hip: 7680 u8 / 15360 4-bit)
  int64_t row_begin;
  const int32_t* row_order;  // nullable: dequeue order of the rows (e.g. heaviest first)
  bool out_by_slot;          // output row = dequeue slot (dps_cct_topk_rows), else x - row_begin
  // split rows: dequeue slots r < n_pieces are row PIECES -- target tiles
  // [piece_t0[r], piece_t1[r]) of row row_order[r] -- whose ranked entries go
  // to piece_*[r] with no zero-score fill (dps_topk_merge completes the rows)
  int64_t n_pieces;
  const int32_t* piece_t0;
  const int32_t* piece_t1;
  int32_t* piece_idx;
  int64_t* piece_cnt;
  double* piece_score;
  int64_t n_rows;
  int k;
  int32_t* out_idx;
  int64_t* out_cnt;
  double* out_score;
  unsigned long long* counter;
  bool dbuf;                 // two alternating stage buffers (W <= 16384) or one
  int ablate;                // profiling aid (DPATHSIM_ABLATE, -DDPS_PROFILE builds only):
                             // 1 no LDS adds, 2 no candidate scoring, 4 no scatter
  // venue skipping (lean kernel, dps_venue_skip in dpathsim.h; all null = off):
  // s[v] the global-walk weights, hv_slot[v] the heavy-venue slot or -1,
  // hv_c[label * n_hv + slot] = C[y, venue of slot] for target label(y)
  const int64_t* s;
  const int32_t* hv_slot;
  const uint16_t* hv_c;
  int n_hv;
  // W = 16384 (4-bit counters) only: the same C^T cut at 8192 with u8-counter
  // entries (null = off): a tile whose 4-bit bound exceeds 15 runs as its two
  // u8 halves instead of wide 4-bit passes
  const uint32_t* h_off;
  const uint32_t* h_ent;
  const uint32_t* h_maxc;
  int64_t T8;
  // optimistic 4-bit passes (dps_cct1.hip, kOptMax): per-bucket count sums of
  // the 16384-target tiles (dps_ct_tiles_sums); null = tiles above 15 split
  const uint32_t* tile_sum;
  // symmetric mode (lean kernel, dps_cct_sym): M[x,y] = M[y,x],
  // so a pair is scanned once.  Row x in tile a = label(x) >> shift:
  //   sym = 1  band pass: tiles [a - band, a + band] only;
  //   sym = 2  rest pass: "strong" rows (row_strong[x]) scan tiles > a + band
  //            only, with their band list's k-th entry (seed_*[x * k + k - 1])
  //            as the threshold floor, and list what beats it (no zero fill);
  //            the others scan every tile from scratch.  A pair with tile(y) >
  //            a + band is seen by x alone: x hands it to y as a record
  //            (rec_y = y, rec_x = x, rec_m = M) when its score reaches
  //            tau_emit[label(y)] (a lower bound of y's k-th score; +inf for
  //            rows that scan everything themselves); tau_blk[label >> 11] is
  //            the minimum of tau_emit over 2048 labels (the epilogue filter),
  //            tau_tile over a tile (which tiles a row may not skip).  Rows
  //            run in descending label order and, when done, raise tau_emit
  //            to their own k-th score; the last row of a block (of a tile)
  //            recomputes tau_blk (tau_tile).  Every value any reader sees is
  //            a lower bound of the row's final k-th score.
  int sym;
  int band;
  const uint8_t* row_strong;
  const int32_t* seed_idx;
  const double* seed_score;
  float* tau_emit;
  float* tau_blk;
  float* tau_tile;           // min tau_emit over each tile (tile skipping)
  uint32_t* blk_done;        // rows finished per 2048-label block (rest pass)
  uint32_t* tile_done;       // blocks finished per tile
  int32_t* rec_y;
  int32_t* rec_x;
  int32_t* rec_m;
  unsigned long long* rec_n;
  int64_t rec_cap;
};

// Lean one-wave kernel for W = 8192 (dps_cct1.hip).
int cct1_launch(const CctParams& p, hipStream_t st);

namespace {

// Profiling aids (DPATHSIM_ABLATE=8 event counters, =16 shader-clock phase
// timers) are compiled in only with -DDPS_PROFILE; the production build keeps
// their state out of the register budget.
#ifdef DPS_PROFILE
constexpr bool kProfile = true;
#else
constexpr bool kProfile = false;
#endif
// The device-assert debug build (make debug, -DDPS_DEBUG).
#ifdef DPS_DEBUG
constexpr bool kDebug = true;
#else
constexpr bool kDebug = false;
#endif

// Waves per workgroup NW is a template parameter: 4 (256 threads) for tiles
// up to W = 32768, 8 (512 threads) for W = 65536, so that a CU always holds 16
// waves (4 workgroups x 32 KB or 2 x 64 KB of accumulators).
#ifndef DPS_KU
#define DPS_KU 4
#endif
constexpr int kU = DPS_KU;          // 16-B chunk loads in flight per lane
#ifndef DPS_EPIU
#define DPS_EPIU 4
#endif
constexpr int kEpiU = DPS_EPIU;    // epilogue blocks read per trip
constexpr int kQ = 2 * kWave;       // per-wave candidate queue (label, M) capacity

typedef unsigned short us2 __attribute__((ext_vector_type(2)));

// ---- top-k order: score desc, then ORIGINAL target index asc ---------------
__device__ __forceinline__ bool better(double s1, int y1, double s2, int y2) {
  return s1 > s2 || (s1 == s2 && y1 < y2);
}

// Integer threshold: a lower bound on m* = the smallest m >= 0 with
// fl(2m / den) >= kth, equal to m* in practice.  Every target y with g[y] >= g0
// has gx + g[y] >= den := gx + g0, so (rounding is monotone) fl(2M/(gx+g[y])) <=
// fl(2M/den), and m -> fl(2m/den) is nondecreasing: a target with M < m* scores
// strictly below kth and cannot enter the top-k, ties included.
// fl(2m*/den) >= kth gives 2m*/den >= kth*(1 - 2^-53), i.e. m* >= r*(1 - 2^-53)
// with r = kth*den/2; the computed r' = kth*den*0.5*(1 - 2^-50) (two roundings)
// is below r*(1 - 2^-53), so ceil(r') <= m*.  Two multiplies, no division.
__device__ __forceinline__ int mneed_lo(double kth, int64_t den) {
  if (kth <= 0.0 || den <= 0) return 0;
  const double r = kth * static_cast<double>(den) * (0.5 * (1.0 - 0x1p-50));
  if (r >= 2147483000.0) return INT32_MAX;
  return static_cast<int>(ceil(r));
}

// The same threshold in fp32 (the per-stage thresholds and tile bounds are
// pure filters: any value <= m* is sound, a smaller one only admits more
// candidates to the exact fp64 score).  Inputs: kth as float, den as the sum of
// two non-negative int64 converted by i64_f32 (relative error <= 3*2^-24 each).
// Every rounding here is round-to-nearest, so the computed product is at most
// r*(1 + 7*2^-24) with r = kth*den/2; the factor (1 - 2^-19) (exact in fp32)
// brings it below r*(1 - 2^-53) <= m*, hence ceil() <= m* as before.
__device__ __forceinline__ float i64_f32(int64_t v) {   // v >= 0
  const uint64_t u = static_cast<uint64_t>(v);
  return __uint2float_rn(static_cast<uint32_t>(u >> 32)) * 4294967296.0f +
         __uint2float_rn(static_cast<uint32_t>(u));
}
// (selects, not branches: den is per lane in the segment thresholds)
__device__ __forceinline__ int mneed_lo32(float kth, float den) {
  const float r = kth * den * (0.5f * (1.0f - 0x1p-19f));
  const int m = static_cast<int>(ceilf(fminf(fmaxf(r, 0.0f), 2147483000.0f)));
  return !(kth > 0.0f) || !(den > 0.0f) ? 0 : r >= 2147483000.0f ? INT32_MAX : m;
}

// Register-resident sorted top-k of one wave: rank r*64 + lane in slot r.
template <int KPL>
struct TopK {
  double s[KPL];
  int y[KPL];
  int m[KPL];
  int k;
  int filled;
  double kth_s;
  int kth_y;
  bool floored;

  __device__ void init(int k_) {
#pragma unroll
    for (int r = 0; r < KPL; ++r) { s[r] = -1.0; y[r] = INT_MAX; m[r] = 0; }
    k = k_;
    filled = 0;
    kth_s = -1.0;
    kth_y = INT_MAX;
    floored = false;
  }
  __device__ bool full() const { return filled == k || floored; }
  // Threshold floor (symmetric rest pass): the row's k-th score so far is at
  // least (fs, fy) -- its band list's k-th -- although this list starts empty;
  // kth stays at the floor until k entries beat it.
  __device__ void set_floor(double fs, int fy) {
    kth_s = fs;
    kth_y = fy;
    floored = true;
  }
  // Insert a candidate known to beat the k-th entry (wave-uniform arguments).
  __device__ void insert(double cs, int cy, int cm) {
    const int lane = lane_id();
    int pos = 0;
#pragma unroll
    for (int r = 0; r < KPL; ++r) {
      // slots r*64 + lane < k that rank above the candidate: ballots of one
      // compare each (a ballot of a compound predicate materialises it)
      const int nv = k - r * kWave;
      const uint64_t valid = nv >= kWave ? ~0ull : nv <= 0 ? 0ull : ((1ull << nv) - 1ull);
      const uint64_t b = ballot(s[r] > cs) | (ballot(s[r] == cs) & ballot(y[r] < cy));
      pos += __popcll(b & valid);
    }
    double us[KPL];
    int uy[KPL], um[KPL];
#pragma unroll
    for (int r = 0; r < KPL; ++r) {
      // lane i <- lane i-1 with a DPP wave shift (no LDS round trip)
      const uint64_t sb = static_cast<uint64_t>(__double_as_longlong(s[r]));
      const int lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(sb), 0x138, 0xF, 0xF, false);
      const int hi = __builtin_amdgcn_update_dpp(0, static_cast<int>(sb >> 32), 0x138, 0xF, 0xF, false);
      us[r] = __longlong_as_double(static_cast<long long>(
          (static_cast<uint64_t>(static_cast<uint32_t>(hi)) << 32) | static_cast<uint32_t>(lo)));
      uy[r] = __builtin_amdgcn_update_dpp(0, y[r], 0x138, 0xF, 0xF, false);
      um[r] = __builtin_amdgcn_update_dpp(0, m[r], 0x138, 0xF, 0xF, false);
      if (r > 0) {
        // lane 0 <- lane 63 of the register below.  The readlanes run with the
        // whole wave active: under `lane == 0` an -O1 build (registers spilled
        // to scratch, the loop not unrolled) reloaded s[r - 1] for lane 0 only
        // and read lane 63's stale copy (round 6, k > 64 in the debug build)
        const double ps = readlane(s[r - 1], kWave - 1);
        const int py = readlane(y[r - 1], kWave - 1), pm = readlane(m[r - 1], kWave - 1);
        us[r] = lane == 0 ? ps : us[r];
        uy[r] = lane == 0 ? py : uy[r];
        um[r] = lane == 0 ? pm : um[r];
      }
    }
#pragma unroll
    for (int r = 0; r < KPL; ++r) {     // selects, not branches
      const int slot = r * kWave + lane;
      const bool up = slot > pos, at = slot == pos;
      s[r] = up ? us[r] : at ? cs : s[r];
      y[r] = up ? uy[r] : at ? cy : y[r];
      m[r] = up ? um[r] : at ? cm : m[r];
    }
    filled = filled < k ? filled + 1 : k;
    if (floored && filled < k) return;   // the floor stays the threshold
    const int rk = (k - 1) / kWave, lk = (k - 1) % kWave;
#pragma unroll
    for (int r = 0; r < KPL; ++r)
      if (r == rk) { kth_s = readlane(s[r], lk); kth_y = readlane(y[r], lk); }
  }
};


// Up to 64 venues of the row for one tile (lane j = venue g0 + j).
struct Grp {
  uint32_t base; // lane j: lo_j - 4*pre_j, so chunk q of venue j is at base_j + 4q
  int c;         // C[x, v_j]
  int pre;       // exclusive prefix of chunk counts
  int nq;        // total chunks (wave-uniform)
  int nv;        // venues in the group (wave-uniform, <= 64)
};

// wave64 inclusive prefix sum / total of a u32 with DPP row shifts and row
// broadcasts (gfx9 DPP: no LDS round trips).  Lanes shifted in from outside a
// row, or masked off by the row/bank masks, contribute 0.
#define DPS_DPP(v, ctrl, rm, bm) \
  static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), ctrl, rm, bm, false))
__device__ __forceinline__ uint32_t wave_incl_sum_u32(uint32_t x) {
  x += DPS_DPP(x, 0x111, 0xF, 0xF);   // row_shr:1
  x += DPS_DPP(x, 0x112, 0xF, 0xF);   // row_shr:2
  x += DPS_DPP(x, 0x114, 0xF, 0xE);   // row_shr:4
  x += DPS_DPP(x, 0x118, 0xF, 0xC);   // row_shr:8
  x += DPS_DPP(x, 0x142, 0xA, 0xF);   // row_bcast:15
  x += DPS_DPP(x, 0x143, 0xC, 0xF);   // row_bcast:31
  return x;
}
// Total over the wave (wave-uniform result).
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t x) {
  return static_cast<uint32_t>(readlane(static_cast<int>(wave_incl_sum_u32(x)), kWave - 1));
}

__device__ __forceinline__ void grp_set(Grp& G, uint32_t lo, uint32_t hi, int c, int nv) {
  G.c = c;
  const int nch = static_cast<int>((hi - lo) >> 2);
  const int inc = static_cast<int>(wave_incl_sum_u32(static_cast<uint32_t>(nch)));
  G.pre = inc - nch;
  G.base = lo - 4u * static_cast<uint32_t>(G.pre);
  G.nq = readlane(inc, kWave - 1);
  G.nv = nv;
}

constexpr int kSmallGroup = 8;

// Venue owning chunk q = the largest j < nv with pre_j <= q.  Small groups:
// compare against the prefix held in SGPRs (sp[]); larger ones: binary search
// over ceil(log2(nv)) shuffle steps.  All lanes must run it.
__device__ __forceinline__ int chunk_venue(const Grp& G, const int (&sp)[kSmallGroup], int q) {
  if (G.nv <= kSmallGroup) {
    int j = 0;
#pragma unroll
    for (int jj = 1; jj < kSmallGroup; ++jj) j += (jj < G.nv && q >= sp[jj]) ? 1 : 0;
    return j;
  }
  int step = 1;
  while (step * 2 < G.nv) step *= 2;
  int j = 0;
  for (; step > 0; step >>= 1) {
    const int cand = j + step;
    const int pv = __shfl(G.pre, cand & (kWave - 1), kWave);
    if (cand < G.nv && pv <= q) j = cand;
  }
  return j;
}

// One accumulation pass over one target tile.  A tile whose bound UB fits in
// 8 bits accumulates four targets per dword in one pass (99.8 % of the tiles
// scanned on config3); UB <= 65535 takes two passes over half the tile at 16
// bits, larger bounds four passes at 32 bits.  UB bounds every accumulator of
// the tile, so no lane can carry into its neighbour.
struct Stage {
  Grp G;
  int t;         // tile (< 2^31: tile offsets are 32-bit)
  int lnp;       // log2(number of passes): 0 u8, 1 u16, 2 u32
  int pass;
  int nb;        // batches of NW*64*kU chunks (0 under the no-scatter ablation)
  int64_t gq;    // lane s: smallest g of segment s of tile t
};

struct Batch {
  uint4 e[kU];
  int c[kU];
};

// Issue the loads of batch b of stage S: chunk q -> lane (q mod 64*NW) of the
// workgroup, kU chunks per lane.  Each load instruction reads 64 consecutive
// chunks (q0 .. q0+63, q0 wave-uniform).  The venues owning its first and last
// chunk come from two ballots over the venue lanes (pre_j <= q), so they are
// scalars; when they agree (the common case: heavy venues own most chunks) the
// base address and C[x,v] are scalars and the load costs a few VALU.  A load
// straddling a few boundaries resolves each lane's venue with one readlane
// compare per boundary; many boundaries take the shuffle search of
// chunk_venue().  Loads past the stage's last chunk are skipped (uniform) and
// marked dead (c = 0).
constexpr int kFewBoundaries = 3;

template <int NW>
__device__ __forceinline__ void issue(Stage& S, int b, const uint32_t* __restrict__ ent,
                                      int wave, int lane, Batch& B, bool no_add,
                                      int p_ablate = 0, unsigned long long* p_counter = nullptr) {
  const bool vl = lane < S.G.nv;
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const int q0 = b * (NW * kWave * kU) + u * (NW * kWave) + wave * kWave;   // wave-uniform
    B.c[u] = 0;
    B.e[u] = make_uint4(0, 0, 0, 0);
    if (q0 >= S.G.nq) continue;
    const int q = q0 + lane;
    const bool live = q < S.G.nq;
    const int qlast = min(q0 + kWave - 1, S.G.nq - 1);
    const int jlo = __popcll(ballot(vl && S.G.pre <= q0)) - 1;
    const int jhi = __popcll(ballot(vl && S.G.pre <= qlast)) - 1;
    uint32_t bj = readlane(S.G.base, jlo);
    int cj = readlane(S.G.c, jlo);
    if ((kProfile && (p_ablate & 8)) && lane == 0) atomicAdd(p_counter + (jhi == jlo ? 20 : 21), 1ull);
    if (jhi > jlo) {
      if (jhi - jlo <= kFewBoundaries) {
        for (int j = jlo + 1; j <= jhi; ++j) {   // wave-uniform loop
          const bool ge = q >= readlane(S.G.pre, j);
          const uint32_t bn = readlane(S.G.base, j);
          const int cn = readlane(S.G.c, j);
          bj = ge ? bn : bj;
          cj = ge ? cn : cj;
        }
      } else {
        int sp[kSmallGroup];
#pragma unroll
        for (int jj = 0; jj < kSmallGroup; ++jj) sp[jj] = readlane(S.G.pre, jj);
        const int j = chunk_venue(S.G, sp, q);
        bj = static_cast<uint32_t>(__shfl(static_cast<int>(S.G.base), j, kWave));
        cj = __shfl(S.G.c, j, kWave);
      }
    }
    B.e[u] = *reinterpret_cast<const uint4*>(ent + (live ? bj + 4u * static_cast<uint32_t>(q) : 0u));
    B.c[u] = live && !no_add ? cj : 0;
  }
}

// One entry (tile-local label yl, count ce) into the u16 / u32 accumulators.
__device__ __forceinline__ void acc_add(uint32_t* acc, uint32_t yl, uint32_t ce, int c, int lnp,
                                        int pass, int shift) {
  const uint32_t val = static_cast<uint32_t>(c) * ce;
  if (val == 0) return;
  uint32_t* dst;
  uint32_t add;
  if (lnp == 0) {
    dst = acc + (yl >> 2);
    add = val << ((yl & 3u) << 3);
  } else {
    if (static_cast<int>(yl >> (shift - lnp)) != pass) return;
    const uint32_t local = yl & ((1u << (shift - lnp)) - 1u);
    if (lnp == 1) {
      dst = acc + (local >> 1);
      add = val << ((local & 1u) << 4);
    } else {
      dst = acc + local;
      add = val;
    }
  }
  __hip_atomic_fetch_add(dst, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// A word of entries: two 16-bit entries (label << 3 | e) when P16 (padding
// codes e >= 6 at label % 4 == 3 add nothing here), else one 32-bit entry
// (C << 16 | label).
__device__ __forceinline__ void acc_add_p16(uint32_t* acc, uint32_t h, int c, int lnp, int pass,
                                            int shift) {
  const uint32_t e = h & 7u, yl = (h >> 3) & 0x1FFFu;
  if ((yl & 3u) == 3u && e >= 6u) return;
  acc_add(acc, yl, 1u << e, c, lnp, pass, shift);
}
template <bool P16>
__device__ __forceinline__ void acc_add_word(uint32_t* acc, uint32_t w, int c, int lnp, int pass,
                                             int shift) {
  if constexpr (P16) {
    acc_add_p16(acc, w & 0xFFFFu, c, lnp, pass, shift);
    acc_add_p16(acc, w >> 16, c, lnp, pass, shift);
  } else {
    acc_add(acc, w & 0xFFFFu, w >> 16, c, lnp, pass, shift);
  }
}

template <bool P16>
__device__ __forceinline__ void scatter(const Batch& B, const Stage& S, uint32_t* acc, int shift) {
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    if (B.c[u] == 0) continue;
    acc_add_word<P16>(acc, B.e[u].x, B.c[u], S.lnp, S.pass, shift);
    acc_add_word<P16>(acc, B.e[u].y, B.c[u], S.lnp, S.pass, shift);
    acc_add_word<P16>(acc, B.e[u].z, B.c[u], S.lnp, S.pass, shift);
    acc_add_word<P16>(acc, B.e[u].w, B.c[u], S.lnp, S.pass, shift);
  }
}

typedef __attribute__((address_space(3))) uint32_t lds_u32;

// u8 accumulation (UB <= 255): one LDS byte per target, four per dword.  The
// entry's low 16 bits are the tile-local label: bits [2, shift) pick the dword,
// bits [0, 2) the byte, so the LDS address is buf | (e & lab_mask) (buf is
// W-aligned) and the byte shift is (e << 3) mod 32 -- five VALU per entry and no
// branch.  Padding entries carry C = 0 (they add 0 to a spread-out dword).
__device__ __forceinline__ void add_u8(uint32_t buf, uint32_t e, uint32_t c, uint32_t lab_mask) {
  const uint32_t val = __umul24(c, e >> 16);
  const uint32_t add = val << ((e << 3) & 31u);
  __hip_atomic_fetch_add(reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(buf | (e & lab_mask))),
                         add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The same for a word of two 16-bit entries (label << 3) | e (W <= 8192): the
// entry's low five bits are 8*(label % 4) + e, exactly the shift that puts
// C * 2^e into the target's byte, and v_lshlrev reads only those five bits --
// no multiply, no mask: seven VALU per word.  Padding groups add C * 2^32 to
// one dword, i.e. nothing (dps_tiles.hip).
__device__ __forceinline__ void add_u8_p16(uint32_t buf, uint32_t w, uint32_t c,
                                           uint32_t lab_mask) {
  const uint32_t alo = c << (w & 31u);
  const uint32_t ahi = c << ((w >> 16) & 31u);
  __hip_atomic_fetch_add(
      reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(buf | ((w >> 3) & lab_mask))), alo,
      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __hip_atomic_fetch_add(
      reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(buf | ((w >> 19) & lab_mask))), ahi,
      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <bool P16>
__device__ __forceinline__ void add_u8_word(uint32_t buf, uint32_t w, uint32_t c,
                                            uint32_t lab_mask) {
  if constexpr (P16) add_u8_p16(buf, w, c, lab_mask);
  else add_u8(buf, w, c, lab_mask);
}

template <bool P16>
__device__ __forceinline__ void scatter_u8(const Batch& B, uint32_t buf, uint32_t lab_mask) {
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const uint32_t c = static_cast<uint32_t>(B.c[u]);
    // dead chunk (beyond the stage's last): skipped, although C = 0 would add
    // nothing -- its lanes all point at entry 0, and 64 adds to one LDS dword
    // serialise (branch-free: 115 -> 489 ms)
    if (c == 0) continue;
    add_u8_word<P16>(buf, B.e[u].x, c, lab_mask);
    add_u8_word<P16>(buf, B.e[u].y, c, lab_mask);
    add_u8_word<P16>(buf, B.e[u].z, c, lab_mask);
    add_u8_word<P16>(buf, B.e[u].w, c, lab_mask);
  }
}

template <bool P16>
__device__ __forceinline__ void scatter_any(const Batch& B, const Stage& S, uint32_t* acc,
                                            uint32_t buf, uint32_t lab_mask, int shift) {
  if (S.lnp == 0) scatter_u8<P16>(B, buf, lab_mask);
  else scatter<P16>(B, S, acc, shift);
}

__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Per-wave candidate queue in LDS: targets that passed the integer threshold
// wait here so their exact scores (two global loads each) are computed 64 at
// a time -- one memory round trip per batch instead of per find.
struct CandQ {
  int* lab;   // [kQ] label
  int* m;     // [kQ] M
  int n;      // wave-uniform fill
};

// Exact score of the first n (<= 64) queued candidates; insert those that beat
// the wave's k-th entry and the shared tau; drop them from the queue.
template <int KPL>
__device__ __forceinline__ void flush(const CctParams& p, CandQ& Q, TopK<KPL>& top, int n,
                                      int64_t gx, double tau_sh, int lane) {
  wave_lds_fence();
  bool cand = lane < n;
  int M = 0, yo = 0;
  double sc = 0.0;
  if (cand) {
    const int64_t label = Q.lab[lane];
    M = Q.m[lane];
    yo = p.t_perm ? p.t_perm[label] : static_cast<int>(label);
    const int64_t den = gx + p.g_t[label];
    sc = static_cast<double>(2 * static_cast<int64_t>(M)) / static_cast<double>(den);
    cand = sc >= tau_sh && better(sc, yo, top.kth_s, top.kth_y);
  }
  int tl = 0, tm = 0;                      // keep the unprocessed tail at the front
  const bool mv = lane + n < Q.n;
  if (mv) { tl = Q.lab[lane + n]; tm = Q.m[lane + n]; }
  wave_lds_fence();
  if (mv) { Q.lab[lane] = tl; Q.m[lane] = tm; }
  Q.n -= n;
  uint64_t mask = ballot(cand);
  if ((kProfile && (p.ablate & 8)) && lane == 0) {       // counters: flushes, candidates, passers
    atomicAdd(p.counter + 1, 1ull);
    atomicAdd(p.counter + 2, static_cast<unsigned long long>(n));
    atomicAdd(p.counter + 3, static_cast<unsigned long long>(__popcll(mask)));
  }
  while (mask) {
    const int srcl = __ffsll(static_cast<long long>(mask)) - 1;
    mask &= mask - 1;
    const double cs = readlane(sc, srcl);
    const int cy = readlane(yo, srcl);
    if (!better(cs, cy, top.kth_s, top.kth_y)) continue;
    top.insert(cs, cy, readlane(M, srcl));
  }
}

// True if some accumulator of the 16-byte block may reach m (exact for 16 and
// 32 bits; for 8 bits exact when m <= 128, else any byte >= 128).
__device__ __forceinline__ bool block_any(uint4 a, uint32_t m, int lnp) {
  if (lnp == 0) {
    if (m > 128u) return ((a.x | a.y | a.z | a.w) & 0x80808080u) != 0;
    const uint32_t k = (128u - m) * 0x01010101u;
    const uint32_t f = (a.x | ((a.x & 0x7F7F7F7Fu) + k)) | (a.y | ((a.y & 0x7F7F7F7Fu) + k)) |
                       (a.z | ((a.z & 0x7F7F7F7Fu) + k)) | (a.w | ((a.w & 0x7F7F7F7Fu) + k));
    return (f & 0x80808080u) != 0;
  }
  if (lnp == 1) {
    const us2 mx = __builtin_elementwise_max(
        __builtin_elementwise_max(__builtin_bit_cast(us2, a.x), __builtin_bit_cast(us2, a.y)),
        __builtin_elementwise_max(__builtin_bit_cast(us2, a.z), __builtin_bit_cast(us2, a.w)));
    return (mx.x > mx.y ? mx.x : mx.y) >= m;
  }
  return max(max(a.x, a.y), max(a.z, a.w)) >= m;
}

// Per-byte flags (bit 7 of each byte) of a packed u8 dword: byte >= m, exact
// for 1 <= m <= 255 (no carry crosses a byte: low7 + 128 - m <= 254).  Both
// forms are computed and selected, branch-free; kA/kB are the broadcast bytes
// 128 - m and 256 - m, lowm = (m <= 128).
__device__ __forceinline__ uint32_t ge_u8(uint32_t a, uint32_t kA, uint32_t kB, bool lowm) {
  const uint32_t lo = a & 0x7F7F7F7Fu;
  const uint32_t rA = a | (lo + kA);
  const uint32_t rB = a & (lo + kB);
  return (lowm ? rA : rB) & 0x80808080u;
}
// u8 stage epilogue: scan + zero the wave's quarter.  One iteration covers 1024
// targets (64 lanes x 16), which is exactly one threshold segment, so the
// threshold m is wave-uniform.  A block passes a cheap prefilter when some byte
// has a bit at or above the highest power of two <= m; only then are its targets
// compared exactly (SWAR) and the flagged ones appended to the wave's queue
// lane-parallel (one round per candidate of the busiest lane).
template <int KPL, int NW>
__device__ __forceinline__ void epilogue_u8(const CctParams& p, uint32_t* acc, TopK<KPL>& top,
                                            CandQ& Q, const Stage& S, int wave, int lane,
                                            int nbuf, int seg_shift, int64_t x_lab, int64_t gx,
                                            double tau_sh, int mseg) {
  const int qd = nbuf / NW;
  const int end = (wave + 1) * qd;
  const int64_t tile_base = static_cast<int64_t>(S.t) << p.shift;
  const bool score = !kProfile || (p.ablate & 2) == 0;
  const int64_t xr64 = x_lab - tile_base;
  const int xrel = (xr64 >= 0 && xr64 < (int64_t(1) << p.shift)) ? static_cast<int>(xr64) : -64;
  // one iteration: the 16-byte block of each lane (1024 targets, one segment)
  auto block = [&](uint4 a, int b0) {
    const int b = b0 + lane * 4;
    const uint32_t m = static_cast<uint32_t>(readlane(mseg, (b0 << 2) >> seg_shift));
    if (m > 255u || !score) return;                          // no u8 count reaches m
    const uint32_t pm = (0x100u - (0x80000000u >> __builtin_clz(m))) * 0x01010101u;
    const uint32_t any = (a.x | a.y | a.z | a.w) & pm;
    if ((kProfile && (p.ablate & 8)) && lane == 0) atomicAdd(p.counter + 16, 1ull);   // iterations scanned
    if (!ballot(any != 0)) return;
    if ((kProfile && (p.ablate & 8)) && lane == 0) atomicAdd(p.counter + 17, 1ull);   // prefilter passes
    const uint32_t kA = __builtin_amdgcn_perm(0u, 128u - m, 0u);   // byte 0 broadcast
    const uint32_t kB = __builtin_amdgcn_perm(0u, 256u - m, 0u);
    const bool lowm = m <= 128u;
    // target (4*dw + byte) of the block -> bit 8*byte + 7 - dw
    uint32_t F = ge_u8(a.x, kA, kB, lowm) | (ge_u8(a.y, kA, kB, lowm) >> 1) |
                 (ge_u8(a.z, kA, kB, lowm) >> 2) | (ge_u8(a.w, kA, kB, lowm) >> 3);
    const int i0 = b << 2;                                     // first target of the block
    const int rel = xrel - i0;                                 // the source itself never counts
    if (rel >= 0 && rel < 16) F &= ~(1u << ((rel & 3) * 8 + 7 - (rel >> 2)));
    if (!ballot(F != 0)) return;
    if ((kProfile && (p.ablate & 8)) && lane == 0) atomicAdd(p.counter + 18, 1ull);   // exact passes
    wave_lds_fence();
    for (;;) {
      const bool has = F != 0;
      const uint64_t mk = ballot(has);
      if (!mk) break;
      if ((kProfile && (p.ablate & 8)) && lane == 0) atomicAdd(p.counter + 19, 1ull); // extraction rounds
      if (has) {
        const int bit = __builtin_ctz(F);
        F &= F - 1;
        const int byte = bit >> 3, dw = 7 - (bit & 7);
        const uint32_t w01 = (dw & 1) ? a.y : a.x;
        const uint32_t w23 = (dw & 1) ? a.w : a.z;
        const uint32_t wv = (dw & 2) ? w23 : w01;
        const int pos = Q.n + mbcnt(mk);
        Q.lab[pos] = static_cast<int>(tile_base + i0 + dw * 4 + byte);
        Q.m[pos] = static_cast<int>((wv >> (byte * 8)) & 0xFFu);
      }
      Q.n += __popcll(mk);
      if (Q.n >= kWave) flush<KPL>(p, Q, top, kWave, gx, tau_sh, lane);
    }
  };
  if (qd % (kWave * 4 * kEpiU) == 0) {
    // whole iterations, kEpiU per trip: all blocks are read (and zeroed) before
    // any is judged, so one LDS latency covers kEpiU segments
    for (int b0 = wave * qd; b0 < end; b0 += kWave * 4 * kEpiU) {
      const int b = b0 + lane * 4;
      uint4 a[kEpiU];
#pragma unroll
      for (int i = 0; i < kEpiU; ++i) a[i] = *reinterpret_cast<const uint4*>(acc + b + i * kWave * 4);
#pragma unroll
      for (int i = 0; i < kEpiU; ++i)
        *reinterpret_cast<uint4*>(acc + b + i * kWave * 4) = make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < kEpiU; ++i) block(a[i], b0 + i * kWave * 4);
    }
    return;
  }
  for (int b0 = wave * qd; b0 < end; b0 += kWave * 4) {
    const int b = b0 + lane * 4;
    uint4 a = make_uint4(0, 0, 0, 0);
    if (b < end) {
      a = *reinterpret_cast<const uint4*>(acc + b);
      *reinterpret_cast<uint4*>(acc + b) = make_uint4(0, 0, 0, 0);
    }
    block(a, b0);
  }
}

// Scan + zero this wave's quarter of the stage's accumulator; queue the
// targets whose M reaches their segment's threshold.
// This lane's segment threshold for stage S: targets of segment `lane` need
// M >= mseg to possibly reach the larger of tau_sh and the wave's k-th score.
template <int KPL>
__device__ __forceinline__ int stage_mseg(const TopK<KPL>& top, const Stage& S, float gxf,
                                          double tau_sh) {
  double tau_w = tau_sh;
  if (top.full() && top.kth_s > tau_w) tau_w = top.kth_s;
  int mseg = 1;
  if (tau_w > 0.0) {
    const int mn = mneed_lo32(static_cast<float>(tau_w), gxf + i64_f32(S.gq));
    mseg = mn > 1 ? mn : 1;
  }
  return mseg;
}

template <int KPL, int NW>
__device__ __forceinline__ void epilogue(const CctParams& p, uint32_t* acc, TopK<KPL>& top,
                                         CandQ& Q, const Stage& S, int wave, int lane, int nbuf,
                                         int seg_shift, int64_t x_lab, int64_t gx,
                                         double tau_sh, int mseg) {
  if (S.lnp == 0) {
    epilogue_u8<KPL, NW>(p, acc, top, Q, S, wave, lane, nbuf, seg_shift, x_lab, gx, tau_sh, mseg);
    return;
  }
  const int qd = nbuf / NW;
  const int end = (wave + 1) * qd;
  const int lnp = S.lnp;
  const int tpd_shift = 2 - lnp;                     // log2(targets per dword)
  const int bits = 8 << lnp;
  const uint32_t vmask = lnp == 2 ? 0xFFFFFFFFu : ((1u << bits) - 1u);
  const int64_t tile_base = static_cast<int64_t>(S.t) << p.shift;
  const int pass_base = S.pass << (p.shift - lnp);
  const bool score = !kProfile || (p.ablate & 2) == 0;
  for (int b0 = wave * qd; b0 < end; b0 += kWave * 4) {
    const int b = b0 + lane * 4;
    uint4 a = make_uint4(0, 0, 0, 0);
    if (b < end) {
      a = *reinterpret_cast<const uint4*>(acc + b);
      *reinterpret_cast<uint4*>(acc + b) = make_uint4(0, 0, 0, 0);
    }
    const int i0 = pass_base + (b << tpd_shift);            // first target of the block
    const int ms = __shfl(mseg, (i0 >> seg_shift) & (kWave - 1), kWave);
    const uint32_t m = static_cast<uint32_t>(ms);
    const bool any = block_any(a, m, lnp);
    if (!score || !ballot(any)) continue;
    wave_lds_fence();
#pragma unroll 1
    for (int v = 0; v < (16 >> lnp); ++v) {
      const int di = v >> tpd_shift;
      const uint32_t wv = di == 0 ? a.x : di == 1 ? a.y : di == 2 ? a.z : a.w;
      const uint32_t M = (wv >> ((v & ((1 << tpd_shift) - 1)) * bits)) & vmask;
      const int64_t label = tile_base + i0 + v;
      const bool cand = any && M >= m && label != x_lab;
      const uint64_t mk = ballot(cand);
      if (!mk) continue;
      if (cand) {
        const int pos = Q.n + mbcnt(mk);
        Q.lab[pos] = static_cast<int>(label);
        Q.m[pos] = static_cast<int>(M);
      }
      Q.n += __popcll(mk);
      if (Q.n >= kWave) flush<KPL>(p, Q, top, kWave, gx, tau_sh, lane);
    }
  }
}

}  // namespace
}  // namespace dps
