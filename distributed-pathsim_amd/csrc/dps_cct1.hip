// ★ Hot path, lean variant: the fused C.C^T + fp64 score + top-k kernel for the
// bench shape -- tiles of W = 8192 targets with 16-bit entries, one wave per
// source row, any row degree, k <= 256 (replaces
// metapath_pairwise_walk DPathSim_APVPA.py:90-109, the score :51-52 and the
// target loop :18-22,36).  Same operands, same results (bit for bit) as
// k_cct_topk in dps_cct.hip; what differs is how the per-tile work is driven:
//
//   tile walk   the row's tile bounds UB[t] = sum_v C[x,v] * maxc[v,t] are
//               computed 64 tiles at a time, lane = tile (coalesced maxc
//               reads, no per-tile wave reduction), together with each tile's
//               smallest g.  A 64-bit mask of the tiles that can still hold a
//               top-k target is refiltered with one ballot whenever the row's
//               k-th score tau rises; the next tile is the mask's lowest bit
//               (scalar), so skipped tiles cost nothing and no load sits on
//               the path from one tile to the next.
//   pipeline    the next tile's bucket bounds are loaded one stage ahead and
//               its first chunk batch is issued before this stage's epilogue,
//               as in k_cct_topk; no barrier, no LDS round trip for tau.
//   epilogue    the exact byte compare uses the single-form SWAR test when the
//               segment threshold m <= 128 (every case that matters); the
//               self-exclusion runs only in the source's own tile.
//
// Skipping a tile is sound for the same reason as in k_cct_topk: UB bounds
// every M of the tile and mneed_lo32(tau, gx + gmin_t) is at most the
// smallest M whose score can reach tau (ties included).
//
// Venue skipping (HV, the row-sum denominator only): every target y has
// g[y] = sum_u C[y,u] s_u, so for a venue set H of row x,
// M_H(y) = sum_{h in H} a_h b_h <= rho_H * g[y] with a = C[x,.], b = C[y,.] and
// rho_H = max_{h in H} a_h / s_h.  Once the row's top-k is full (k-th score
// tau), the heavy venues with 2 a_h <= tau s_h form H: their buckets are no
// longer scattered, and score(y) >= tau needs
//   M_Q(y) >= tau (gx + g[y]) / 2 - rho_H g[y]     (Q = the other venues),
// whose right side does not decrease in g[y] (rho_H <= tau / 2), so the
// segment's smallest g gives a sound per-segment threshold.  A target that
// passes gets its exact M = M_Q + sum_{h in H} a_h C[y,h] from the dense
// heavy-venue table hv_c (one cache line per target) before it is scored.
// The heavy venues hold most of C^T's entries (config3: half of the chunks a
// row scatters), and once every venue of a row is in H no target can reach
// tau at all (score < 2 rho_H <= tau), so the row ends.
// Three 64-chunk loads per batch (not the general kernel's four): with the
// candidate queue in VGPRs it keeps the kernel within 96 VGPRs, 5 waves per SIMD.
#ifndef DPS_KU
#define DPS_KU 3
#endif
#include "dps_cct_dev.hpp"

#include <cstdlib>
#include <type_traits>

namespace dps {
namespace {

// Two tile formats share this kernel (template F, dps_tiles.hip):
//   F = 1  W = 8192 targets, 16-bit entries (l << 3) | e, packed u8 counters;
//   F = 2  W = 16384 targets, 16-bit entries (l << 2) | e, packed 4-bit counters.
// Both keep one tile's counters in 8 KiB of LDS per wave (2048 dwords), and in
// both the entry's low five bits are the add's shift and (entry >> 3) masked
// to a dword is its LDS byte address, so the scatter is the same code.  The
// 4-bit counters halve the accumulator passes per row.  A tile whose bound
// exceeds 15 runs as its two halves from a companion W = 8192 (u8) tile set
// when the caller provides one ("dual", p.h_ent): each half scatters only its
// own entries, through the same branch-free path; without it the tile takes
// wide 4-bit passes (u8 / u16 / u32 counters, one entry at a time).
// A kernel parameter read where it is used -- an s_load from the kernarg
// segment each time (the kernel's only argument is the CctParams, at offset
// 0) -- instead of being held in SGPRs, or spilled to VGPR lanes, across the
// whole row loop: for the fields only the per-row code needs.  The asm
// launders the base so the loads cannot be hoisted back out of the loop.
// (Taking p's address instead would copy the struct to scratch.)
template <class T>
__device__ __forceinline__ T kcold_at(size_t off) {
  typedef const __attribute__((address_space(4))) char* kb;
  kb base = (kb)(__builtin_amdgcn_kernarg_segment_ptr());
  asm volatile("" : "+s"(base));
  return *reinterpret_cast<const __attribute__((address_space(4))) T*>(base + off);
}
#define kcold(field) kcold_at<decltype(CctParams::field)>(offsetof(CctParams, field))

constexpr int kAcc1 = 2048;                   // accumulator dwords (8 KiB)
constexpr uint32_t kLabMask1 = 0x1FFCu;       // (entry >> 3) & mask = dword byte address
template <int F> struct Fmt;
template <> struct Fmt<1> {
  static constexpr int S = 13;                // log2 W
  static constexpr int BITS = 8;              // counter bits of the base pass
  static constexpr uint32_t UB0 = 0xFFu;      // largest bound of the base pass
};
template <> struct Fmt<2> {
  static constexpr int S = 14;
  static constexpr int BITS = 4;
  static constexpr uint32_t UB0 = 0xFu;
};
// Tile geometry (round 6).  One-wave workgroups with 8 KiB of LDS run 18 per
// CU, not 20: the LDS a CU gives its workgroups is ~150 KiB in 512-byte
// granules (tools/ubench/resident.hip: 18 resident at 7712..8192 bytes, 20 at
// 7680; the hot launch's wave stamps showed 512 of its 5120 workgroups
// starting only at the end, tools/wave_times.py), so the T15 layout cuts a
// tile to 15 / 16 of the power-of-two width -- 15360 targets in 4-bit
// counters, 7680 in u8, 7680 bytes either way -- and 20 waves fit a CU.  A
// tile's eight threshold segments (= epilogue trips) are then 960 bytes, read
// by lanes 0..59 (lanes 60..63 re-read lane 59's bytes and are masked off).
template <int F, bool T15>
struct Geo {
  static constexpr int W = (T15 ? 15 : 16) * (F == 1 ? 512 : 1024);   // targets per tile
  static constexpr int TPD = F == 1 ? 4 : 8;          // targets per accumulator dword
  static constexpr int SEGW = W / 8;                  // targets per segment (= per trip)
  static constexpr int TRIP_DW = SEGW / TPD;          // dwords per trip: 256 or 240
  static constexpr int LANES = TRIP_DW / 4;           // lanes reading 16 B of a trip
  static constexpr int ACC_DW = 8 * TRIP_DW;          // accumulator dwords: 2048 or 1920
};
// Lane l's first dword within a trip (lanes past the trip's reuse the last one).
template <int F, bool T15>
__device__ __forceinline__ int trip_lane(int lane) {
  return (Geo<F, T15>::LANES < kWave && lane >= Geo<F, T15>::LANES ? Geo<F, T15>::LANES - 1 : lane) * 4;
}
template <int F, bool T15>
__device__ __forceinline__ uint32_t trip_mask(int lane) {
  return Geo<F, T15>::LANES < kWave && lane >= Geo<F, T15>::LANES ? 0u : ~0u;
}

// Knobs, swept on the full config3 launch at W = 16384 (profiles/r03/ab7-ab9):
// epilogue blocks per trip 1 / 2 = 72.3 / 73.2 ms; boundary selects before the
// counting path 4 / 8 / 16 = 72.3 / 73.2 / 73.8 ms; flush the candidate queue
// once the list is full at 8 / 12 / 16 / 24 / 32 / 48 candidates (earlier
// flushes raise tau sooner) -- together 69.3-70.0 against 73.1 ms.
#ifndef DPS_EPI1
#define DPS_EPI1 1
#endif
#ifndef DPS_FLUSH_AT
#define DPS_FLUSH_AT 12   // queued candidates that trigger a flush once the list is full
#endif
constexpr int kEpi1 = DPS_EPI1;                // epilogue blocks read per trip

// Optimistic 4-bit pass check: the digit sum of the nibbles of each half of
// the 8 KiB accumulator (blocks 0-3 = targets 0..8191, blocks 4-7; one
// v_dot8_u32_u4 with 0x11111111 per dword) equals exp_a / exp_b exactly when
// no count of that half carried out of its nibble (see kOptMax).  Returns the
// epilogue's block mask: bits 0-3 when half a is good, 4-7 when half b is.
__device__ __forceinline__ uint32_t opt_check(const uint32_t* acc, uint32_t exp, int lane) {
  const uint32_t exp_a = exp & 0xFFFFu, exp_b = exp >> 16;   // 0xFFFF: saturated, never equal
  uint32_t sa = 0, sb = 0;
#pragma unroll 2
  for (int b0 = 0; b0 < kAcc1 / 2; b0 += kWave * 4) {
    const uint4 a = *reinterpret_cast<const uint4*>(acc + b0 + lane * 4);
    const uint4 b = *reinterpret_cast<const uint4*>(acc + kAcc1 / 2 + b0 + lane * 4);
    sa = __builtin_amdgcn_udot8(a.x, 0x11111111u, sa, false);
    sa = __builtin_amdgcn_udot8(a.y, 0x11111111u, sa, false);
    sa = __builtin_amdgcn_udot8(a.z, 0x11111111u, sa, false);
    sa = __builtin_amdgcn_udot8(a.w, 0x11111111u, sa, false);
    sb = __builtin_amdgcn_udot8(b.x, 0x11111111u, sb, false);
    sb = __builtin_amdgcn_udot8(b.y, 0x11111111u, sb, false);
    sb = __builtin_amdgcn_udot8(b.z, 0x11111111u, sb, false);
    sb = __builtin_amdgcn_udot8(b.w, 0x11111111u, sb, false);
  }
  return (exp_a != 0xFFFFu && wave_sum_u32(sa) == exp_a ? 0x0Fu : 0u) |
         (exp_b != 0xFFFFu && wave_sum_u32(sb) == exp_b ? 0xF0u : 0u);
}

// Zero the kEpi1 KiB of accumulator an epilogue trip has just read (dwords
// b0..).  (ds_write_addtid_b32 zeroes 1.46x faster in isolation,
// tools/ubench/addtid.hip, but did not move the kernel: DESIGN.md §6.)
template <int F, bool T15>
__device__ __forceinline__ void zero_trip(uint32_t* acc, int b0, int lane) {
#pragma unroll
  for (int i = 0; i < kEpi1; ++i)
    *reinterpret_cast<uint4*>(acc + b0 + i * Geo<F, T15>::TRIP_DW + trip_lane<F, T15>(lane)) =
        make_uint4(0, 0, 0, 0);
}


// Symmetric rest pass: the bounds other rows raise are read with plain loads
// (any value read is a valid bound; an atomic load would wait for every
// outstanding load of the wave, the prefetched chunks included).
__device__ __forceinline__ float ld_fresh(const float* a) { return *a; }
__device__ __forceinline__ float wave_min_f32(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fminf(v, __shfl_xor(v, off, kWave));
  return v;
}

// 64 consecutive tiles of one row: lane l describes tile w0 + l.
struct Win1 {
  int w0;          // first tile of the window (wave-uniform)
  uint32_t ub;     // lane: UB of the tile (0xFFFFFFFF = unbounded)
  uint32_t hb;     // dual (F = 2 with companion u8 tiles): the bounds of the
                   // tile's two u8 halves 2t, 2t+1, 16 bits each (kHalfSat =
                   // 65535 or more: the half takes the tile's own bound)
  float gmf;       // lane: smallest g of the tile, as float
  uint64_t live;   // tiles not yet visited that may hold a top-k target
  uint64_t ykeep;  // symmetric rest pass: tiles that may hold a pair to hand on
  float tau;       // tau the mask was last filtered with (rounded: a missed tiny rise
                   // only postpones a refilter)
};
constexpr uint32_t kHalfSat = 0xFFFFu;

// UB of tiles w0 + lane over all d venues of the row (lane j of c / vT holds
// venue j of the first 64; rows with more venues reload them per group) and,
// when dual, the bounds of the tile's two companion u8 halves in the same
// loop (hb, see Win1): computed here lane-parallel, once per window, instead
// of one wave reduction with an exposed h_maxc load per split tile in the
// stage transition (round 4; the load's vmcnt wait also drained the next
// stage's just-issued chunk loads).
__device__ __forceinline__ uint32_t win_ub(const CctParams& p, int w0, int t_end, int64_t pb, int d,
                                           int c, uint32_t vT, uint32_t vT8, bool dual, int lane,
                                           uint32_t& hb) {
  const int t = w0 + lane;
  const bool in = t < t_end;
  hb = kHalfSat | (kHalfSat << 16);
  if (!p.use_bounds) return 0xFFFFFFFFu;        // no tile bounds: every tile, 32-bit passes
  uint64_t acc = 0, ha = 0, hz = 0;
  const bool in_a = dual && in;                  // half 2t always exists when t does
  const bool in_b = dual && in && 2 * t + 1 < p.T8;
  for (int g0 = 0; g0 < d; g0 += kWave) {
    int cg = c;
    uint32_t vg = vT, vg8 = vT8;
    if (g0 > 0) {
      const int j = g0 + lane;
      cg = j < d ? kcold(c_val)[pb + j] : 0;
      const uint32_t vj = j < d ? static_cast<uint32_t>(kcold(c_col)[pb + j]) : 0u;
      vg = vj * static_cast<uint32_t>(p.T);
      vg8 = dual ? vj * static_cast<uint32_t>(p.T8) : 0u;
    }
    const int nj = d - g0 < kWave ? d - g0 : kWave;
#pragma unroll 4
    for (int j = 0; j < nj; ++j) {
      const uint32_t cj = readlane(static_cast<unsigned>(cg), j);
      const uint32_t vj = readlane(vg, j);
      const uint32_t mx = in ? p.tile_maxc[vj + static_cast<uint32_t>(t)] : 0u;
      acc += static_cast<uint64_t>(cj) * mx;
      if (dual) {
        const uint32_t vj8 = readlane(vg8, j) + 2u * static_cast<uint32_t>(t);
        const uint32_t ma = in_a ? p.h_maxc[vj8] : 0u;
        const uint32_t mb = in_b ? p.h_maxc[vj8 + 1u] : 0u;
        ha += static_cast<uint64_t>(cj) * ma;
        hz += static_cast<uint64_t>(cj) * mb;
      }
    }
  }
  if (dual) {
    const uint32_t a = ha >= kHalfSat ? kHalfSat : static_cast<uint32_t>(ha);
    const uint32_t b = hz >= kHalfSat ? kHalfSat : static_cast<uint32_t>(hz);
    hb = a | (b << 16);
  }
  return acc >= 0xFFFFFFFFull ? 0xFFFFFFFFu : static_cast<uint32_t>(acc);
}

// Tiles of the window whose bound reaches mneed(tau) (all of them while tau <= 0).
__device__ __forceinline__ uint64_t win_pass(const Win1& w, double tau, float gxf) {
  if (!(tau > 0.0)) return ~0ull;
  const int mn = mneed_lo32(static_cast<float>(tau), gxf + w.gmf);
  return ballot(w.ub >= static_cast<uint32_t>(mn));
}

template <bool SY>
__device__ __forceinline__ void win_load(const CctParams& p, Win1& w, int w0, int t_lo, int t_end,
                                         int64_t pb, int d, int c, uint32_t vT, uint32_t vT8,
                                         bool dual, int lane, double tau, float gxf, int far) {
  w.w0 = w0;
  const int t = w0 + lane;
  w.gmf = t < t_end ? i64_f32(p.tile_gmin[t]) : 0.0f;
  w.ub = win_ub(p, w0, t_end, pb, d, c, vT, vT8, dual, lane, w.hb);
  w.ykeep = 0;
  if (SY && far != INT_MAX) {
    // a far tile stays while its bound reaches the smallest count any of its
    // targets needs (tau_tile: min tau_emit over the tile)
    const float ty = t >= far && t < t_end ? ld_fresh(p.tau_tile + t) : __builtin_inff();
    w.ykeep = ballot(ty < __builtin_inff() &&
                     w.ub >= static_cast<uint32_t>(max(mneed_lo32(ty, gxf + w.gmf), 1)));
  }
  w.live = ballot(t >= t_lo && t < t_end && w.ub > 0) & (win_pass(w, tau, gxf) | w.ykeep);
  w.tau = static_cast<float>(tau);
}

// Next tile to process (-1: none left); slides the window as needed.
template <bool SY>
__device__ __forceinline__ int next_tile(const CctParams& p, Win1& w, int t_end, int64_t pb, int d,
                                         int c, uint32_t vT, uint32_t vT8, bool dual, int lane,
                                         double tau, float gxf, uint32_t& ub_t, uint32_t& hb_t,
                                         int far) {
  for (;;) {
    if (w.live) {
      const int b = __builtin_ctzll(w.live);
      w.live &= w.live - 1;
      ub_t = readlane(w.ub, b);
      if (dual) hb_t = readlane(w.hb, b);
      return w.w0 + b;
    }
    if (w.w0 + kWave >= t_end) return -1;
    win_load<SY>(p, w, w.w0 + kWave, w.w0 + kWave, t_end, pb, d, c, vT, vT8, dual, lane, tau, gxf,
                 far);
  }
}

// Bucket bounds of one tile (lane j < 64: venue j) and the smallest g of each of
// its 8 threshold segments (lane s < 8), loaded one stage ahead.
struct Pend1 {
  int t;         // tile (u8h: a half tile of the companion W = 8192 set)
  uint32_t ub;
  bool u8h;
  bool opt;      // optimistic 4-bit pass over a tile whose bound exceeds 15 (see kOptMax)
  uint32_t hb;   // opt: the tile's two half bounds (Win1::hb), for the redo
  uint32_t lo, hi;
  uint32_t mx;   // venue skipping: max C[y,v] over the tile's targets (lane = venue)
  uint32_t hs;   // opt: the count sums of the venue's buckets in the two u8 halves
                 // (tile_sum of the companion tiles), 16 bits each, saturated
  int64_t gs;
  float tb;      // symmetric rest pass, far tile: lane s < 8, min tau_emit over segment s
};

// Optimistic 4-bit passes (round 4).  A 16384-target tile whose 4-bit bound
// exceeds 15 used to run as its two u8 halves (two accumulator passes, 24 % of
// all passes on config3), but the bound is loose: most such tiles have no
// target with 16 or more paths (tools/sim_overflow.py).  Such a tile now takes
// ONE 4-bit pass, and a nibble that overflowed is detected exactly before
// anything is read from the accumulator: a count c >= 16 carries into the next
// nibble (or out of the dword), which lowers the sum of the nibble digits by 15
// (16) per carry, so the digit sum of a half's 4 KiB of counters
// (v_dot8_u32_u4 against 0x11111111, one VALU per dword) equals
// sum_{v scattered} C[x,v] * tile_sum[v, half] -- the sum of the half's counts
// -- if and only if none of its counts reached 16.  Carries never cross the
// halves (a dword holds 8 consecutive labels), so each half is judged alone: a
// good half goes through the epilogue, a bad one is cleared and queued to run
// again as its u8 half tile (the old path).  Results are exact either way.
// Tiles whose bound exceeds kOptMax, rows with more than 64 venues and the
// symmetric mode split as before.
#ifndef DPS_OPT_MAX
#define DPS_OPT_MAX 255
#endif
#ifndef DPS_OPT_INEPI
#define DPS_OPT_INEPI 0   // 1: judge each half inside the epilogue (no separate read)
#endif
constexpr uint32_t kOptMax = DPS_OPT_MAX;   // 0 = off
constexpr uint32_t kOptSumMax = 0xFFFFu;    // bucket sums above this: no opt pass

template <int F, bool HV, bool SY, bool T15>
__device__ __forceinline__ void pend_load(const CctParams& p, Pend1& P, int t, uint32_t ub, bool u8h,
                                          int d0, uint32_t vT, uint32_t vT8, int lane, int far,
                                          bool opt = false, uint32_t hb = 0) {
  P.t = t;
  P.ub = ub;
  P.u8h = u8h;
  P.opt = opt;
  P.hb = hb;
  P.lo = P.hi = 0;
  P.mx = 0;
  P.gs = 0;
  P.tb = __builtin_inff();
  if (t < 0) return;
  if (lane < d0) {
    const uint32_t* off = u8h ? p.h_off : p.tile_off;
    const uint32_t b = (u8h ? vT8 : vT) + static_cast<uint32_t>(t);
    P.lo = off[b];
    P.hi = off[b + 1u];
    if (HV) P.mx = p.use_bounds ? (u8h ? p.h_maxc : p.tile_maxc)[b] : 0xFFFFu;
    P.hs = 0;
    if (opt) {                  // the tile's halves 2t, 2t+1 in the companion set
      const uint32_t b8 = vT8 + 2u * static_cast<uint32_t>(t);
      const uint32_t sa = p.tile_sum[b8];
      const uint32_t sb = 2 * t + 1 < p.T8 ? p.tile_sum[b8 + 1u] : 0u;
      P.hs = (sa < kOptSumMax ? sa : kOptSumMax) | ((sb < kOptSumMax ? sb : kOptSumMax) << 16);
    }
  }
  if (lane < 8) {
    const int64_t w = u8h ? Geo<1, T15>::W : Geo<F, T15>::W;
    const int64_t sw = u8h ? Geo<1, T15>::SEGW : Geo<F, T15>::SEGW;
    const int64_t i = static_cast<int64_t>(t) * w + static_cast<int64_t>(lane) * sw;
    P.gs = p.g_t[i < p.n_targets ? i : p.n_targets - 1];
    if (SY && (u8h ? (t >> 1) : t) >= far) P.tb = ld_fresh(p.tau_blk + ((i < p.n_targets ? i : p.n_targets - 1) >> 11));
  }
}

struct Stage1 {
  Stage S;       // chunk group, tile, pass mode (shared helpers' view)
  float gsf;     // lane s < 8: smallest g of segment s, as float
  float tbf;     // lane s < 8: symmetric rest pass, min tau_emit of segment s (inf: none)
  bool u8h;      // a u8 half tile of the companion set (F = 2, dual)
  bool opt;      // optimistic 4-bit pass (Pend1::opt)
  uint32_t hb;   // opt: half bounds for the redo
  uint32_t exp;  // opt: each half's digit sum when none of its counts reached 16, 16 bits
                 // each (saturated at 0xFFFF: the check then fails, both halves run again)
  int ubh;       // venue skipping: sum_{h in H} C[x,h] * maxc[h, tile] >= M_H of any target
};

// hm: the venue lanes (H) whose buckets this stage skips (venue skipping).
template <int F>
__device__ __forceinline__ void stage_make(Stage1& X, const Pend1& P, int c, int d0, uint64_t hm,
                                           int lane) {
  X.S.t = P.t;
  X.u8h = P.u8h;
  X.opt = P.opt;
  X.hb = P.hb;
  // log2 of the passes: counters of BITS << lnp bits must hold the bound
  if (F == 1 || P.u8h) X.S.lnp = P.ub <= 0xFFu ? 0 : P.ub <= 0xFFFFu ? 1 : 2;
  else X.S.lnp = P.ub <= 0xFu || P.opt ? 0 : P.ub <= 0xFFu ? 1 : P.ub <= 0xFFFFu ? 2 : 3;
  X.S.pass = 0;
  const bool skip = (hm >> lane) & 1ull;          // an H venue's bucket is not scattered
  grp_set(X.S.G, P.lo, skip ? P.lo : P.hi, c, d0);
  X.exp = 0;
  if (P.opt) {
    // sum of the counts the scatter adds to each half: C[x,v] * (count sum of
    // the venue's bucket in that half) over the scattered venues; above 8192 *
    // 15 some count must exceed 15, so the check is made to fail (saturated
    // sums do the same)
    auto part = [&](uint32_t sm) -> uint32_t {
      const uint64_t pr64 = skip ? 0ull : static_cast<uint64_t>(c) * sm;
      return sm >= kOptSumMax || pr64 > 0xFFFFull ? 0xFFFFu : static_cast<uint32_t>(pr64);
    };
    const uint32_t ea = wave_sum_u32(part(P.hs & 0xFFFFu));
    const uint32_t eb = wave_sum_u32(part(P.hs >> 16));
    X.exp = (ea < 0xFFFFu ? ea : 0xFFFFu) | ((eb < 0xFFFFu ? eb : 0xFFFFu) << 16);
  }
  X.ubh = 0;
  if (hm) {
    // c, mx <= 65535: the product fits 32 bits; a product beyond 16 bits makes
    // the bound useless (saturate upward: a larger ubh is always sound)
    const uint32_t pr = skip ? static_cast<uint32_t>(c) * P.mx : 0u;
    X.ubh = ballot(pr > 0xFFFFu) ? 0x3FFFFFFF : static_cast<int>(wave_sum_u32(pr));
  }
  X.S.nb = (X.S.G.nq + kWave * kU - 1) / (kWave * kU);
  X.S.gq = 0;
  X.gsf = i64_f32(P.gs);
  X.tbf = P.tb;
}

// Per-byte flags (bit 7) of a packed u8 dword: byte >= m, for 1 <= m <= 128.
__device__ __forceinline__ uint32_t ge_u8_lo(uint32_t a, uint32_t kA) {
  return (a | ((a & 0x7F7F7F7Fu) + kA)) & 0x80808080u;
}

// Order the row's first 64 venues by their total bucket size, smallest first,
// so a stage's small buckets sit together at the front of the flattened chunk
// range (one vector load) and the large ones fill whole fast loads.
template <bool HV>
__device__ __forceinline__ void sort_venues(const CctParams& p, int d0, int lane, int& c, uint32_t& vT,
                                            int& v) {
  int key = INT_MAX;
  if (lane < d0) {
    const uint32_t n = p.tile_off[vT + static_cast<uint32_t>(p.T)] - p.tile_off[vT];
    key = static_cast<int>((n < (1u << 24) ? n : (1u << 24) - 1u) << 6) | lane;
  }
  // (the network's lane masks rebuilt per row: hoisted, they held 42 SGPRs for
  // the whole kernel and pushed ~250 SGPR spills into the stage loop)
  const int src = wave_bitonic_sort(key, opaque_lane(lane)) & (kWave - 1);
  c = __shfl(c, src, kWave);
  vT = static_cast<uint32_t>(__shfl(static_cast<int>(vT), src, kWave));
  if (HV) v = __shfl(v, src, kWave);
}

// Venue skipping state of venue lane j in one VGPR: the bits of an fp32 upper
// bound of C[x,v] / s_v with the low 7 mantissa bits replaced by slot + 1
// (kHvNone, a NaN, = not a heavy venue: it compares false with every
// threshold, so the H ballot is one compare).  Rounding the ratio up to a
// multiple of 2^-16 relative first keeps the packed value an upper bound.
constexpr uint32_t kHvSlot = 0x7Fu;
constexpr uint32_t kHvNone = 0xFFFFFFFFu;
__device__ __forceinline__ uint32_t hv_pack(float ratio_up, int slot) {
  if (slot < 0) return kHvNone;
  const uint32_t b = (__float_as_uint(ratio_up) & ~kHvSlot) + (kHvSlot + 1u);
  return b | static_cast<uint32_t>(slot + 1);
}
__device__ __forceinline__ float hv_ratio(uint32_t hv) { return __uint_as_float(hv); }

// Per-row state every candidate flush needs: the wave-uniform work counts
// (candidates completed from the heavy-venue table, counter[3]; profiling
// build: candidates scored and inserted, counter[15..16]) and, in the rest pass
// of the symmetric mode, the row and the first tile whose pairs it hands on.
struct RowAux {
  uint32_t ver = 0, cand = 0, ins = 0;
  uint32_t redo = 0;            // optimistic 4-bit passes that overflowed (counter[4])
  uint32_t u8h = 0, wide = 0;   // profiling build: half-tile and wide passes
  // profiling build: epilogue blocks by outcome (counter[19..23]): threshold
  // above the counter width, prefilter empty, exact test empty, with
  // candidates; and candidate extraction rounds
  uint32_t bk[5] = {0, 0, 0, 0, 0};
  // profiling build: passes by the stage's chunk count (bucket edges 0 / 16 /
  // 64 / 128 / 192 / 384 / 768), their chunks and their epilogue cycles
  // (counter[24..31], [32..39], [40..47])
  uint32_t nqh[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t nqc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t nqe[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int x = 0;               // source row (ordinal)
  int far = INT_MAX;       // sym = 2: targets in tiles >= far may go to records
};

// Symmetric rest pass, end of row x (label lx): raise tau_emit[lx] to the row's
// own k-th score (strong rows; it only grows: the band k-th is its floor), then
// count the row done in its 2048-label block; the block's last row recomputes
// tau_blk, the tile's last block tau_tile.  No fences: every value another
// wave may read, stale or fresh, is a valid lower bound (a stale read only
// loosens a filter), and only the counters must be exact (device atomics).
template <int KPL>
__device__ __forceinline__ void sym_publish(const CctParams& p, int64_t lx, bool strong,
                                            const TopK<KPL>& top, int lane) {
  if (strong && top.full() && lane == 0) p.tau_emit[lx] = __double2float_rd(top.kth_s);
  const int64_t b = lx >> 11;
  const int64_t bsz = p.n_targets - (b << 11) < 2048 ? p.n_targets - (b << 11) : 2048;
  uint32_t done = 0;
  if (lane == 0)
    done = __hip_atomic_fetch_add(p.blk_done + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  done = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(done)));
  if (done != static_cast<uint32_t>(bsz)) return;
  float mn = __builtin_inff();
  for (int64_t i = lane; i < bsz; i += kWave) mn = fminf(mn, ld_fresh(p.tau_emit + (b << 11) + i));
  mn = wave_min_f32(mn);
  if (lane == 0) p.tau_blk[b] = mn;
  const int64_t t = lx >> p.shift;
  const int per = 1 << (p.shift - 11);                 // blocks per tile
  const int64_t b0 = t << (p.shift - 11);
  const int64_t nbt_all = (p.n_targets + 2047) >> 11;
  const int nbt = static_cast<int>(nbt_all - b0 < per ? nbt_all - b0 : per);
  uint32_t tdone = 0;
  if (lane == 0)
    tdone = __hip_atomic_fetch_add(p.tile_done + t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  tdone = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(tdone)));
  if (tdone != static_cast<uint32_t>(nbt)) return;
  const float tb = lane < nbt ? ld_fresh(p.tau_blk + b0 + lane) : __builtin_inff();
  const float tm = wave_min_f32(tb);
  if (lane == 0) p.tau_tile[t] = tm;
}

// Candidate queue in VGPRs (no LDS: the wave's 8 KB of LDS is all
// accumulator, so 20 waves fit a CU): slot s lives in lane s % 64, register
// s / 64.  Appends come 64 lanes at a time while n < 64, so n < 128.
struct VQ {
  int lab0, m0;   // slots 0..63
  int lab1, m1;   // slots 64..127
  int n;          // wave-uniform fill
};

// Append the candidates of the lanes in mk (this lane's (lab, m) if set) at
// slots n, n + 1, ...: a forward permute sends each to lane slot % 64; lanes
// without a candidate send theirs to a lane outside the receiving window.
__device__ __forceinline__ void vq_push(VQ& Q, bool has, int lab, int m, uint64_t mk, int lane) {
  const int cnt = __popcll(mk);
  const int pos = Q.n + mbcnt(mk);
  const int dst = has ? (pos & (kWave - 1)) : ((Q.n - 1) & (kWave - 1));
  const int plab = __builtin_amdgcn_ds_permute(dst << 2, lab);
  const int pm = __builtin_amdgcn_ds_permute(dst << 2, m);
  const bool recv = cnt >= kWave || ((lane - Q.n) & (kWave - 1)) < cnt;
  const bool hi = lane < Q.n;                     // wrapped past slot 63
  if (recv && !hi) { Q.lab0 = plab; Q.m0 = pm; }
  if (recv && hi) { Q.lab1 = plab; Q.m1 = pm; }
  Q.n += cnt;
}

// Exact score of the first n (<= 64) queued candidates; insert those that beat
// the k-th entry; drop them from the queue (n == 64 moves slots 64.. down).
// Venue skipping: the queued counts miss the venues of hm (the H of the
// stages that queued them); their exact share sum_{h in H} C[x,h] * C[y,h]
// comes from the heavy-venue table (lane h holds C[x,h] in c and the venue's
// table slot in the low bits of hv, see hv_pack).
template <int KPL, bool HV, bool SY>
__device__ __forceinline__ void vq_flush(const CctParams& p, VQ& Q, TopK<KPL>& top, int n,
                                         int64_t gx, int lane, int c, uint32_t hv, uint64_t hm,
                                         RowAux& ra) {
  if constexpr (!SY) {
    // branch-free: every lane scores (lanes past n read target 0, in bounds,
    // and are masked out), so no exec-mask branches around the loads and the
    // division; the better-than-k-th test is three ballots of one compare each
    const int lab = lane < n ? Q.lab0 : 0;
    int M = Q.m0;
    ra.cand += static_cast<uint32_t>(n);
    if (HV && hm) {
      ra.ver += static_cast<uint32_t>(n);
      const uint16_t* row = p.hv_c + static_cast<int64_t>(lab) * p.n_hv;
      for (uint64_t m = hm; m; m &= m - 1) {          // wave-uniform, |H| is small
        const int j = __builtin_ctzll(m);
        const int a = readlane(c, j);
        const int sl = static_cast<int>(readlane(hv, j) & kHvSlot) - 1;
        M += a * static_cast<int>(row[sl]);
      }
    }
    const int yo = p.t_perm ? p.t_perm[lab] : lab;
    const int64_t den = gx + p.g_t[lab];
    const double sc = static_cast<double>(2 * static_cast<int64_t>(M)) / static_cast<double>(den);
    const uint64_t live = n >= kWave ? ~0ull : ((1ull << n) - 1ull);
    uint64_t mask = live & (ballot(sc > top.kth_s) |
                            (ballot(sc == top.kth_s) & ballot(yo < top.kth_y)));
    if (n >= kWave) { Q.lab0 = Q.lab1; Q.m0 = Q.m1; }
    Q.n -= n;
    while (mask) {
      const int srcl = __ffsll(static_cast<long long>(mask)) - 1;
      mask &= mask - 1;
      const double cs = readlane(sc, srcl);
      const int cy = readlane(yo, srcl);
      if (!better(cs, cy, top.kth_s, top.kth_y)) continue;
      ++ra.ins;
      top.insert(cs, cy, readlane(M, srcl));
    }
    return;
  }
  bool cand = lane < n;
  int M = 0, yo = 0;
  double sc = 0.0;
  ra.cand += static_cast<uint32_t>(n);
  if (HV && hm) {
    ra.ver += static_cast<uint32_t>(n);
    const uint16_t* row = p.hv_c + static_cast<int64_t>(cand ? Q.lab0 : 0) * p.n_hv;
    for (uint64_t m = hm; m; m &= m - 1) {          // wave-uniform, |H| is small
      const int j = __builtin_ctzll(m);
      const int a = readlane(c, j);
      const int sl = static_cast<int>(readlane(hv, j) & kHvSlot) - 1;
      if (cand) M += a * static_cast<int>(row[sl]);
    }
  }
  bool emit = false;
  if (cand) {
    const int64_t label = Q.lab0;
    M += Q.m0;
    yo = p.t_perm ? p.t_perm[label] : static_cast<int>(label);
    const int64_t den = gx + p.g_t[label];
    sc = static_cast<double>(2 * static_cast<int64_t>(M)) / static_cast<double>(den);
    // symmetric rest pass: a pair in a far tile can enter y's top-k only
    // through this row (tau_emit <= y's exact band k-th score, rounded down)
    if (SY && (label >> p.shift) >= ra.far) emit = sc >= static_cast<double>(ld_fresh(p.tau_emit + label));
    cand = better(sc, yo, top.kth_s, top.kth_y);
  }
  if (SY && ra.far != INT_MAX) {
    const uint64_t emk = ballot(emit);
    if (emk) {
      unsigned long long base = 0;
      if (lane == 0) base = atomicAdd(p.rec_n, static_cast<unsigned long long>(__popcll(emk)));
      base = (static_cast<unsigned long long>(readlane(static_cast<int>(base >> 32), 0)) << 32) |
             static_cast<uint32_t>(readlane(static_cast<int>(base), 0));
      const unsigned long long slot = base + static_cast<unsigned long long>(mbcnt(emk));
      if (emit && slot < static_cast<unsigned long long>(p.rec_cap)) {
        p.rec_y[slot] = yo;
        p.rec_x[slot] = ra.x;
        p.rec_m[slot] = M;
      }
    }
  }
  if (n >= kWave) { Q.lab0 = Q.lab1; Q.m0 = Q.m1; }
  Q.n -= n;
  uint64_t mask = ballot(cand);
  while (mask) {
    const int srcl = __ffsll(static_cast<long long>(mask)) - 1;
    mask &= mask - 1;
    const double cs = readlane(sc, srcl);
    const int cy = readlane(yo, srcl);
    if (!better(cs, cy, top.kth_s, top.kth_y)) continue;
    ++ra.ins;
    top.insert(cs, cy, readlane(M, srcl));
  }
}

// u16 / u32 pass epilogue (UB > 255, rare): scan + zero the accumulator of
// pass `pass` (2 or 1 targets per dword), queue targets reaching their
// segment's threshold.
template <int F, int KPL, bool HV, bool SY, bool T15>
__device__ __forceinline__ void epi1_wide(const CctParams& p, uint32_t* acc, TopK<KPL>& top, VQ& Q,
                                          const Stage& S, int lane, int64_t x_lab, int64_t gx,
                                          int mseg, int c, uint32_t hv, uint64_t hm, RowAux& ra) {
  using G = Geo<F, T15>;
  const int lnp = S.lnp;
  const int bits = Fmt<F>::BITS << lnp;              // 8..32
  const int tpd_shift = (F == 1 ? 2 : 3) - lnp;      // log2(targets per dword)
  const uint32_t vmask = bits == 32 ? 0xFFFFFFFFu : ((1u << bits) - 1u);
  const int blnp = bits == 8 ? 0 : bits == 16 ? 1 : 2;   // block_any's counter width
  const int64_t tile_base = static_cast<int64_t>(S.t) * G::W;
  const int pass_base = S.pass * (G::W >> lnp);
  // (T15: the 1920-dword accumulator in 1 KiB rows, the last one half used)
  for (int b0 = 0; b0 < G::ACC_DW; b0 += kWave * 4) {
    const int b = b0 + lane * 4;
    const bool in = !T15 || b < G::ACC_DW;
    const uint4 a = in ? *reinterpret_cast<const uint4*>(acc + b) : make_uint4(0, 0, 0, 0);
    if (in) *reinterpret_cast<uint4*>(acc + b) = make_uint4(0, 0, 0, 0);
    const int i0 = pass_base + (b << tpd_shift);     // first target of this lane's 16 bytes
    const int sg = i0 / G::SEGW;                     // its threshold segment
    const uint32_t m = static_cast<uint32_t>(__shfl(mseg, sg & (kWave - 1), kWave));
    const bool any = in && block_any(a, m, blnp);
    if (!ballot(any)) continue;
#pragma unroll 1
    for (int v = 0; v < (128 / bits); ++v) {
      const int di = v >> tpd_shift;
      const uint32_t wv = di == 0 ? a.x : di == 1 ? a.y : di == 2 ? a.z : a.w;
      const uint32_t M = (wv >> ((v & ((1 << tpd_shift) - 1)) * bits)) & vmask;
      const int64_t label = tile_base + i0 + v;
      const bool cand = any && M >= m && label != x_lab;
      const uint64_t mk = ballot(cand);
      if (!mk) continue;
      vq_push(Q, cand, static_cast<int>(label), static_cast<int>(M), mk, lane);
      if (Q.n >= kWave) vq_flush<KPL, HV, SY>(p, Q, top, kWave, gx, lane, c, hv, hm, ra);
    }
  }
}

// 4-bit epilogue over the whole W = 16384 tile: 8 blocks of 2048 targets (one
// threshold segment each; lane l reads dwords 4l..4l+3 of the block = targets
// 32l..32l+31), read and zeroed kEpi1 at a time; candidates queued as in epi1_u8.
// T15: W = 15360, 8 trips of 1920 targets over lanes 0..59.
template <int KPL, bool HV, bool SY, bool T15>
__device__ __forceinline__ void epi1_u4(const CctParams& p, uint32_t* acc, TopK<KPL>& top, VQ& Q,
                                        int t, int lane, int x_lab, int64_t gx, int mseg,
                                        int c, uint32_t hv, uint64_t hm, RowAux& ra,
                                        uint32_t bmask, uint32_t oexp, uint32_t& bad) {
  using G = Geo<2, T15>;
  const int tile_base = t * G::W;                        // labels < 2^31
  const int xr = x_lab - tile_base;
  const bool xin = static_cast<uint32_t>(xr) < static_cast<uint32_t>(G::W);   // the source is a target here
  const int xrel = xin ? xr : 0;
  const uint32_t lmask = trip_mask<2, T15>(lane);        // (all ones unless T15)
  // optimistic pass judged here (oexp != 0, DPS_OPT_INEPI): each half's
  // candidates are held in the queue (no flush) until its digit sum shows no
  // overflowed count; a bad half's candidates are dropped (Q.n back to snap)
  bool hold = oexp != 0u, abort = false;
  uint32_t dsum = 0;
  int snap = Q.n;
  // prefilter masks of the 8 segments, lane s: the nibble bits at or above
  // the highest power of two <= m_s (0 when m_s > 15: no 4-bit count reaches it)
  const uint32_t mu = static_cast<uint32_t>(mseg);
  const uint32_t pmv = mu > 15u ? 0u : (0x10u - (0x80000000u >> __builtin_clz(mu | 1u))) * 0x11111111u;
  auto block = [&](uint4 a, int blk) {
    if (!((bmask >> blk) & 1u)) return;            // overflowed half (optimistic pass)
    const uint32_t pm = static_cast<uint32_t>(readlane(pmv, blk)) & lmask;
    if (kProfile && pm == 0u) {                    // threshold above the counter width
      ++ra.bk[0];
      return;
    }
    if (!ballot(((a.x | a.y | a.z | a.w) & pm) != 0)) {
      if (kProfile) ++ra.bk[1];
      return;
    }
    const uint32_t m = static_cast<uint32_t>(readlane(mseg, blk));
    // target (8*dw + nib) of this lane's 32 -> bit 4*nib + 3 - dw
    // per-nibble flags (bit 3): nibble >= m, 1 <= m <= 15 (no carry leaves a
    // nibble: low3 + 16 - m <= 14); m is wave-uniform, so one branch per block
    // picks the form (per-dword branches cost 2 % of the kernel)
    uint32_t F4;
    if (m <= 8u) {
      const uint32_t K = (8u - m) * 0x11111111u;
      auto ge = [K](uint32_t v) { return (v | ((v & 0x77777777u) + K)) & 0x88888888u; };
      F4 = ge(a.x) | (ge(a.y) >> 1) | (ge(a.z) >> 2) | (ge(a.w) >> 3);
    } else {
      const uint32_t K = (16u - m) * 0x11111111u;
      auto ge = [K](uint32_t v) { return (v & ((v & 0x77777777u) + K)) & 0x88888888u; };
      F4 = ge(a.x) | (ge(a.y) >> 1) | (ge(a.z) >> 2) | (ge(a.w) >> 3);
    }
    F4 &= lmask;

    const int i0 = blk * G::SEGW + (lane << 5);
    if (__builtin_expect(xin, false)) {            // the source itself never counts
      const int rel = xrel - i0;
      if (rel >= 0 && rel < 32) F4 &= ~(1u << ((rel & 7) * 4 + 3 - (rel >> 3)));
    }
    if (!ballot(F4 != 0)) {
      if (kProfile) ++ra.bk[2];
      return;
    }
    if (kProfile) ++ra.bk[3];
    for (;;) {
      const bool has = F4 != 0;
      const uint64_t mk = ballot(has);
      if (!mk) break;
      if (kProfile) ++ra.bk[4];
      // every lane extracts (a lane without a flag gets garbage that vq_push
      // never stores): no exec-mask branch per round
      const int bit = __builtin_ffs(static_cast<int>(F4)) - 1;    // -1 when F4 == 0
      F4 &= F4 - 1;
      const int nib = (bit >> 2) & 7, dw = 3 - (bit & 3);
      const uint32_t w01 = (dw & 1) ? a.y : a.x;
      const uint32_t w23 = (dw & 1) ? a.w : a.z;
      const uint32_t wv = (dw & 2) ? w23 : w01;
      const int lab = tile_base + i0 + dw * 8 + nib;
      const int mv = static_cast<int>((wv >> (nib * 4)) & 0xFu);
      vq_push(Q, has, lab, mv, mk, lane);
      if (Q.n >= kWave) {
        if (hold) {         // an unverified half may not be flushed: give it up
          abort = true;
          return;
        }
        vq_flush<KPL, HV, SY>(p, Q, top, kWave, gx, lane, c, hv, hm, ra);
      }
    }
  };
  // two trips per loop iteration for the top-10 instantiation, four for the
  // two-register top-k (round 5: config3 58.7 vs 60.0 ms with one trip, 58.1
  // vs 58.55 with four; config5 609 vs 624 ms with four instead of two;
  // still one 1 KiB block read per trip)
  constexpr int kTrips = KPL == 1 ? 2 : 4;
  if constexpr (T15) {     // (no optimistic passes: hold is false)
#pragma unroll kTrips
    for (int tr = 0; tr < 8; tr += kEpi1) {
      const int b0 = tr * G::TRIP_DW;
      uint4 a[kEpi1];
#pragma unroll
      for (int i = 0; i < kEpi1; ++i)
        a[i] = *reinterpret_cast<const uint4*>(acc + b0 + i * G::TRIP_DW + trip_lane<2, T15>(lane));
      zero_trip<2, T15>(acc, b0, lane);
#pragma unroll
      for (int i = 0; i < kEpi1; ++i) block(a[i], tr + i);
    }
    return;
  }
#pragma unroll kTrips
  for (int b0 = 0; b0 < kAcc1; b0 += kWave * 4 * kEpi1) {
    uint4 a[kEpi1];
#pragma unroll
    for (int i = 0; i < kEpi1; ++i)
      a[i] = *reinterpret_cast<const uint4*>(acc + b0 + i * kWave * 4 + lane * 4);
    zero_trip<2, T15>(acc, b0, lane);
#pragma unroll
    for (int i = 0; i < kEpi1; ++i) {
      const int blk = (b0 >> 8) + i;
      if (hold) {            // optimistic pass: the digit sum of this half so far
        dsum = __builtin_amdgcn_udot8(a[i].x, 0x11111111u, dsum, false);
        dsum = __builtin_amdgcn_udot8(a[i].y, 0x11111111u, dsum, false);
        dsum = __builtin_amdgcn_udot8(a[i].z, 0x11111111u, dsum, false);
        dsum = __builtin_amdgcn_udot8(a[i].w, 0x11111111u, dsum, false);
      }
      if (!abort) block(a[i], blk);
      if (hold && (blk & 3) == 3) {
        // end of a half: its candidates stand only if no count overflowed
        const uint32_t e = blk == 3 ? (oexp & 0xFFFFu) : (oexp >> 16);
        const bool ok = !abort && e != 0xFFFFu && wave_sum_u32(dsum) == e;
        if (!ok) {
          Q.n = snap;
          bad |= blk == 3 ? 1u : 2u;
        }
        dsum = 0;
        abort = false;
        snap = Q.n;
        if (Q.n >= kWave) {
          hold = false;
          vq_flush<KPL, HV, SY>(p, Q, top, kWave, gx, lane, c, hv, hm, ra);
          hold = true;
          snap = Q.n;
        }
      }
    }
  }
}

// Sparse epilogue (round 6; built, exact, measured slower -- off).  38 % of
// config3's accumulator passes scatter at most 64 chunks (one load; 67 % at most
// 192), yet the dense epilogue reads and zeroes the whole 8 KiB whatever the
// pass scattered (profiles/r06/c/lean_phases.txt: ~11-12 k epilogue cycles per
// pass at 1-16 chunks as at 193-384).  A one-load stage instead exchanges every
// dword its own entries addressed with 0 (ds_wrxchg_rtn_b32, four of a chunk's
// eight entries in flight at once): each nonzero dword comes back to exactly
// one (lane, entry) -- a second entry or a second lane on the same dword gets
// 0 -- so every target of the tile is judged once, and since the accumulator
// was all zero before the stage's scatter, every dword it touched is zero
// again after.  Dead lanes (kDeadChunk) address dword L and judge whatever it
// holds, which is just as exact.  Thresholds per 1 KiB segment (2048 4-bit /
// 1024 u8 targets) come from two wave-uniform words of byte-packed m_s (0:
// above the counter width).  Same digest on all 1 M config3 rows, but 63.7 ms
// against 58.9: the stage's chunks are only in registers until
// the next stage's first loads reuse B, so the sparse stage issues those after
// its epilogue and the scatter then waits out their latency, which the dense
// epilogue hides; holding the chunks or reloading them across the transition
// spills 46-52 VGPRs (84.5 ms).  DPS_SPARSE_LOADS=1 compiles it in.
#ifndef DPS_SPARSE_LOADS
#define DPS_SPARSE_LOADS 0
#endif
constexpr int kSparseLoads = DPS_SPARSE_LOADS;   // 0: dense epilogue only

// Per-target flags of one dword against a lane's own threshold m: 4-bit
// counters (bit 4j+3 for target j: the nibbles spread to bytes, nib + 128 - m
// sets bit 7 exactly when nib >= m, no carry between bytes) or u8 counters
// (bit 8j+7: the two SWAR forms of ge_u8, chosen per lane).  m = 0: none.
__device__ __forceinline__ uint32_t sparse_flags(uint32_t v, uint32_t m, bool u8f) {
  uint32_t f;
  if (u8f) {
    const uint32_t lo = v & 0x7F7F7F7Fu;
    const uint32_t rA = v | (lo + (128u - m) * 0x01010101u);
    const uint32_t rB = v & (lo + ((256u - m) & 0xFFu) * 0x01010101u);
    f = (m <= 128u ? rA : rB) & 0x80808080u;
  } else {
    const uint32_t K = (128u - m) * 0x01010101u;
    const uint32_t lo = v & 0x0F0F0F0Fu, hi = (v >> 4) & 0x0F0F0F0Fu;
    f = (((lo + K) & 0x80808080u) >> 4) | ((hi + K) & 0x80808080u);
  }
  return m != 0u ? f : 0u;
}

template <int KPL, bool HV, bool SY>
__device__ __forceinline__ void epi1_sparse(const CctParams& p, uint32_t* acc, TopK<KPL>& top, VQ& Q,
                                            const uint4 e, int t, bool u8f, int lane,
                                            int x_lab, int64_t gx, int mseg, int c, uint32_t hv,
                                            uint64_t hm, RowAux& ra) {
  const uint32_t mu = static_cast<uint32_t>(mseg);
  const uint32_t ms = mu <= (u8f ? 255u : 15u) ? mu : 0u;
  uint32_t mlo = 0, mhi = 0;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    mlo |= static_cast<uint32_t>(readlane(ms, s)) << (8 * s);
    mhi |= static_cast<uint32_t>(readlane(ms, s + 4)) << (8 * s);
  }
  const int sh = u8f ? Fmt<1>::S : Fmt<2>::S;
  const int tile_base = t << sh;                           // labels < 2^31
  const int tpd_sh = u8f ? 2 : 3;                          // log2(targets per dword)
  const int xr0 = x_lab - tile_base;
  const bool xin = static_cast<uint32_t>(xr0) < (1u << sh);   // the source is a target here
  char* const accb = reinterpret_cast<char*>(acc);
  {
    // two halves of four entries each (four exchanges in flight, then their
    // judging: eight at once held 49 more VGPRs than the kernel has)
#pragma unroll 1
    for (int hf = 0; hf < 2; ++hf) {
      const uint32_t wa = hf ? e.z : e.x;
      const uint32_t wb = hf ? e.w : e.y;
      auto addr = [&](int i) -> uint32_t {                 // the entry's dword, byte address
        const uint32_t w = i < 2 ? wa : wb;
        return ((i & 1) ? (w >> 19) : (w >> 3)) & kLabMask1;
      };
      if ((mlo | mhi) == 0u) {                             // nothing can reach a threshold
#pragma unroll
        for (int i = 0; i < 4; ++i) *reinterpret_cast<uint32_t*>(accb + addr(i)) = 0u;
        continue;
      }
      uint32_t v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        v[i] = __hip_atomic_exchange(reinterpret_cast<uint32_t*>(accb + addr(i)), 0u,
                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      auto flags = [&](int i) -> uint32_t {
        const uint32_t a = addr(i);
        const uint32_t seg = a >> 10;
        const uint32_t mw = seg < 4u ? mlo : mhi;
        uint32_t f = sparse_flags(v[i], (mw >> ((seg & 3u) << 3)) & 0xFFu, u8f);
        if (__builtin_expect(xin, false)) {                // the source itself never counts
          const int rel = xr0 - static_cast<int>((a >> 2) << tpd_sh);
          if (static_cast<uint32_t>(rel) < (1u << tpd_sh)) f &= ~(1u << (u8f ? 8 * rel + 7 : 4 * rel + 3));
        }
        return f;
      };
      const uint32_t any = flags(0) | flags(1) | flags(2) | flags(3);
      if (!ballot(any != 0u)) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        uint32_t f = flags(i);
        if (!ballot(f != 0u)) continue;
        const int lab0 = tile_base + static_cast<int>((addr(i) >> 2) << tpd_sh);
        for (;;) {
          const bool has = f != 0u;
          const uint64_t mk = ballot(has);
          if (!mk) break;
          // every lane extracts (as in epi1_u4: no exec-mask branch per round)
          const int bit = __builtin_ffs(static_cast<int>(f)) - 1;
          f &= f - 1u;
          const int j = u8f ? (bit >> 3) & 3 : (bit >> 2) & 7;
          const int mv = static_cast<int>((v[i] >> (j << (u8f ? 3 : 2))) & (u8f ? 0xFFu : 0xFu));
          vq_push(Q, has, lab0 + j, mv, mk, lane);
          if (Q.n >= kWave) vq_flush<KPL, HV, SY>(p, Q, top, kWave, gx, lane, c, hv, hm, ra);
        }
      }
    }
  }
}

// Wide passes of the 4-bit format (lnp 1..3: u8 / u16 / u32 counters over a
// half / quarter / eighth of the tile per pass), one entry at a time; padding
// codes (e >= 2 at l % 8 == 7) add nothing.
// (T15: passes of 15360 >> lnp targets, found by a division -- a rare path)
template <bool T15>
__device__ __forceinline__ void acc_add4(uint32_t* acc, uint32_t h, int c, int lnp, int pass) {
  const uint32_t e = h & 3u, yl = h >> 2;
  if ((yl & 7u) == 7u && e >= 2u) return;
  uint32_t local;
  if constexpr (T15) {
    const uint32_t pw = 15360u >> lnp, ps = yl / pw;
    if (static_cast<int>(ps) != pass) return;
    local = yl - ps * pw;
  } else {
    if (static_cast<int>(yl >> (14 - lnp)) != pass) return;
    local = yl & ((1u << (14 - lnp)) - 1u);
  }
  const int bits = 4 << lnp;
  const int tpds = 3 - lnp;                          // log2(targets per dword)
  const uint32_t val = static_cast<uint32_t>(c) << e;
  const uint32_t add = val << ((local & ((1u << tpds) - 1u)) * bits);
  __hip_atomic_fetch_add(acc + (local >> tpds), add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// T15 u8-format wide passes (u16 / u32 counters over halves / quarters of a
// 7680-target tile): one entry (label << 3 | e), padding codes add nothing.
__device__ __forceinline__ void acc_add8w(uint32_t* acc, uint32_t h, int c, int lnp, int pass) {
  const uint32_t e = h & 7u, yl = (h >> 3) & 0x1FFFu;
  if ((yl & 3u) == 3u && e >= 6u) return;
  const uint32_t val = static_cast<uint32_t>(c) << e;
  if (val == 0) return;
  const uint32_t pw = 7680u >> lnp, ps = yl / pw;
  if (static_cast<int>(ps) != pass) return;
  const uint32_t local = yl - ps * pw;
  uint32_t* dst = lnp == 1 ? acc + (local >> 1) : acc + local;
  const uint32_t add = lnp == 1 ? val << ((local & 1u) << 4) : val;
  __hip_atomic_fetch_add(dst, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// A batch into the accumulator: the base pass branch-free over the loads
// batch b issued (the u8 / 4-bit adds: dead lanes add 0, see kDeadChunk),
// wide passes entry by entry (u8h: u8-format entries).
template <int F, bool T15>
__device__ __forceinline__ void scatter_f(const Batch& B, const Stage& S, int b, uint32_t* acc,
                                          bool u8h) {
  if (S.lnp == 0) {                                    // u8 or 4-bit base pass
    const int left = S.G.nq - b * (kWave * kU);        // chunks from this batch on (uniform)
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (u * kWave >= left) break;                    // a load issue1 skipped
      const uint32_t c = static_cast<uint32_t>(B.c[u]);
      add_u8_word<true>(0u, B.e[u].x, c, kLabMask1);
      add_u8_word<true>(0u, B.e[u].y, c, kLabMask1);
      add_u8_word<true>(0u, B.e[u].z, c, kLabMask1);
      add_u8_word<true>(0u, B.e[u].w, c, kLabMask1);
    }
    return;
  }
  if (F == 1 || u8h) {                                 // u8-format wide passes
    if constexpr (T15) {
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (B.c[u] == 0) continue;
        const uint32_t w4[4] = {B.e[u].x, B.e[u].y, B.e[u].z, B.e[u].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc_add8w(acc, w4[q] & 0xFFFFu, B.c[u], S.lnp, S.pass);
          acc_add8w(acc, w4[q] >> 16, B.c[u], S.lnp, S.pass);
        }
      }
    } else {
      scatter<true>(B, S, acc, Fmt<1>::S);
    }
    return;
  }
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    if (B.c[u] == 0) continue;
    const uint32_t w4[4] = {B.e[u].x, B.e[u].y, B.e[u].z, B.e[u].w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      acc_add4<T15>(acc, w4[q] & 0xFFFFu, B.c[u], S.lnp, S.pass);
      acc_add4<T15>(acc, w4[q] >> 16, B.c[u], S.lnp, S.pass);
    }
  }
}

// u8 epilogue over the whole tile: 8 blocks of 1024 targets (one threshold
// segment each, lane l reads dwords 4l..4l+3 of the block), read and zeroed 4
// at a time; candidates are queued and scored 64 at a time by flush().
// T15: W = 7680, 8 trips of 960 targets over lanes 0..59.
template <int KPL, bool HV, bool SY, bool T15>
__device__ __forceinline__ void epi1_u8(const CctParams& p, uint32_t* acc, TopK<KPL>& top, VQ& Q,
                                        int t, int lane, int x_lab, int64_t gx, int mseg,
                                        int c, uint32_t hv, uint64_t hm, RowAux& ra) {
  using G = Geo<1, T15>;
  const int tile_base = t * G::W;                        // labels < 2^31
  const int xr = x_lab - tile_base;
  const bool xin = static_cast<uint32_t>(xr) < static_cast<uint32_t>(G::W);   // the source is a target here
  const int xrel = xin ? xr : 0;
  const uint32_t lmask = trip_mask<1, T15>(lane);        // (all ones unless T15)
  // prefilter masks of the 8 segments, lane s (as in epi1_u4; 0 when m_s > 255)
  const uint32_t mu = static_cast<uint32_t>(mseg);
  const uint32_t pmv = mu > 255u ? 0u : (0x100u - (0x80000000u >> __builtin_clz(mu | 1u))) * 0x01010101u;
  auto block = [&](uint4 a, int blk) {
    const uint32_t pm = static_cast<uint32_t>(readlane(pmv, blk)) & lmask;
    if (kProfile && pm == 0u) {                    // threshold above the counter width
      ++ra.bk[0];
      return;
    }
    if (!ballot(((a.x | a.y | a.z | a.w) & pm) != 0)) {
      if (kProfile) ++ra.bk[1];
      return;
    }
    const uint32_t m = static_cast<uint32_t>(readlane(mseg, blk));
    uint32_t F;
    if (m <= 128u) {
      const uint32_t kA = (128u - m) * 0x01010101u;
      F = ge_u8_lo(a.x, kA) | (ge_u8_lo(a.y, kA) >> 1) | (ge_u8_lo(a.z, kA) >> 2) |
          (ge_u8_lo(a.w, kA) >> 3);
    } else {
      const uint32_t kA = (128u - m) * 0x01010101u, kB = (256u - m) * 0x01010101u;
      F = ge_u8(a.x, kA, kB, false) | (ge_u8(a.y, kA, kB, false) >> 1) |
          (ge_u8(a.z, kA, kB, false) >> 2) | (ge_u8(a.w, kA, kB, false) >> 3);
    }
    F &= lmask;
    // target (4*dw + byte) of this lane's 16 -> bit 8*byte + 7 - dw
    const int i0 = blk * G::SEGW + (lane << 4);
    if (__builtin_expect(xin, false)) {           // the source itself never counts
      const int rel = xrel - i0;
      if (rel >= 0 && rel < 16) F &= ~(1u << ((rel & 3) * 8 + 7 - (rel >> 2)));
    }
    if (!ballot(F != 0)) {
      if (kProfile) ++ra.bk[2];
      return;
    }
    if (kProfile) ++ra.bk[3];
    for (;;) {
      const bool has = F != 0;
      const uint64_t mk = ballot(has);
      if (!mk) break;
      if (kProfile) ++ra.bk[4];
      // every lane extracts (as in epi1_u4: no exec-mask branch per round)
      const int bit = __builtin_ffs(static_cast<int>(F)) - 1;    // -1 when F == 0
      F &= F - 1;
      const int byte = (bit >> 3) & 3, dw = 7 - (bit & 7);
      const uint32_t w01 = (dw & 1) ? a.y : a.x;
      const uint32_t w23 = (dw & 1) ? a.w : a.z;
      const uint32_t wv = (dw & 2) ? w23 : w01;
      const int lab = tile_base + i0 + dw * 4 + byte;
      const int mv = static_cast<int>((wv >> (byte * 8)) & 0xFFu);
      vq_push(Q, has, lab, mv, mk, lane);
      if (Q.n >= kWave) vq_flush<KPL, HV, SY>(p, Q, top, kWave, gx, lane, c, hv, hm, ra);
    }
  };
  // four trips per loop iteration (round 5: 58.2 vs 58.8 ms with two)
  if constexpr (T15) {
#pragma unroll 4
    for (int tr = 0; tr < 8; tr += kEpi1) {
      const int b0 = tr * G::TRIP_DW;
      uint4 a[kEpi1];
#pragma unroll
      for (int i = 0; i < kEpi1; ++i)
        a[i] = *reinterpret_cast<const uint4*>(acc + b0 + i * G::TRIP_DW + trip_lane<1, T15>(lane));
      zero_trip<1, T15>(acc, b0, lane);
#pragma unroll
      for (int i = 0; i < kEpi1; ++i) block(a[i], tr + i);
    }
    return;
  }
#pragma unroll 4
  for (int b0 = 0; b0 < kAcc1; b0 += kWave * 4 * kEpi1) {
    uint4 a[kEpi1];
#pragma unroll
    for (int i = 0; i < kEpi1; ++i)
      a[i] = *reinterpret_cast<const uint4*>(acc + b0 + i * kWave * 4 + lane * 4);
    zero_trip<1, T15>(acc, b0, lane);
#pragma unroll
    for (int i = 0; i < kEpi1; ++i) block(a[i], (b0 >> 8) + i);
  }
}

// Issue the loads of batch b of stage S (one wave, NW = 1): chunk q -> lane
// q mod 64, kU loads of 64 consecutive chunks.  The venues owning a load's first
// and last chunk come from two ballots; a load inside one venue has a scalar
// base and C.  Boundaries inside a load are resolved without LDS round trips:
// up to kSel of them by a per-boundary select over readlane'd scalars, more by
// counting the boundaries each lane has passed and fetching base and C from
// that venue's lane with two independent bpermutes.  (kSel swept on the full
// config3 launch: 4 / 8 / 16 = 72.3 / 73.2 / 73.8 ms in round 3; with the
// round-4 register allocation 1 / 2 / 3 / 4 / 6 = 66.45 / 66.5 / 66.65 / 66.86
// / 67.3 ms, profiles/r04/ab/ab4n, ab4o; round 5, after the epilogue and
// flush changes: 1 / 2 / 3 = 59.9 / 60.2 / 60.3 ms, profiles/r05/kab/ab5g.)
#ifndef DPS_KSEL
#define DPS_KSEL 1
#endif
// The chunk a dead lane (past the stage's last chunk) loads instead of a real
// one: lane L's 16-bit entries all address accumulator dword L (h = L << 5 in
// both the u8 and the 4-bit format), and the lane's C is 0, so its adds are
// no-ops on 64 distinct dwords -- no per-lane branch around the adds, and no
// 64-way conflict on one dword (which the branch used to avoid).
__device__ uint4 kDeadChunk[kWave] = {   // (global, not constant: one global_load)
    {0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u}, {0x00200020u, 0x00200020u, 0x00200020u, 0x00200020u},
    {0x00400040u, 0x00400040u, 0x00400040u, 0x00400040u}, {0x00600060u, 0x00600060u, 0x00600060u, 0x00600060u},
    {0x00800080u, 0x00800080u, 0x00800080u, 0x00800080u}, {0x00A000A0u, 0x00A000A0u, 0x00A000A0u, 0x00A000A0u},
    {0x00C000C0u, 0x00C000C0u, 0x00C000C0u, 0x00C000C0u}, {0x00E000E0u, 0x00E000E0u, 0x00E000E0u, 0x00E000E0u},
    {0x01000100u, 0x01000100u, 0x01000100u, 0x01000100u}, {0x01200120u, 0x01200120u, 0x01200120u, 0x01200120u},
    {0x01400140u, 0x01400140u, 0x01400140u, 0x01400140u}, {0x01600160u, 0x01600160u, 0x01600160u, 0x01600160u},
    {0x01800180u, 0x01800180u, 0x01800180u, 0x01800180u}, {0x01A001A0u, 0x01A001A0u, 0x01A001A0u, 0x01A001A0u},
    {0x01C001C0u, 0x01C001C0u, 0x01C001C0u, 0x01C001C0u}, {0x01E001E0u, 0x01E001E0u, 0x01E001E0u, 0x01E001E0u},
    {0x02000200u, 0x02000200u, 0x02000200u, 0x02000200u}, {0x02200220u, 0x02200220u, 0x02200220u, 0x02200220u},
    {0x02400240u, 0x02400240u, 0x02400240u, 0x02400240u}, {0x02600260u, 0x02600260u, 0x02600260u, 0x02600260u},
    {0x02800280u, 0x02800280u, 0x02800280u, 0x02800280u}, {0x02A002A0u, 0x02A002A0u, 0x02A002A0u, 0x02A002A0u},
    {0x02C002C0u, 0x02C002C0u, 0x02C002C0u, 0x02C002C0u}, {0x02E002E0u, 0x02E002E0u, 0x02E002E0u, 0x02E002E0u},
    {0x03000300u, 0x03000300u, 0x03000300u, 0x03000300u}, {0x03200320u, 0x03200320u, 0x03200320u, 0x03200320u},
    {0x03400340u, 0x03400340u, 0x03400340u, 0x03400340u}, {0x03600360u, 0x03600360u, 0x03600360u, 0x03600360u},
    {0x03800380u, 0x03800380u, 0x03800380u, 0x03800380u}, {0x03A003A0u, 0x03A003A0u, 0x03A003A0u, 0x03A003A0u},
    {0x03C003C0u, 0x03C003C0u, 0x03C003C0u, 0x03C003C0u}, {0x03E003E0u, 0x03E003E0u, 0x03E003E0u, 0x03E003E0u},
    {0x04000400u, 0x04000400u, 0x04000400u, 0x04000400u}, {0x04200420u, 0x04200420u, 0x04200420u, 0x04200420u},
    {0x04400440u, 0x04400440u, 0x04400440u, 0x04400440u}, {0x04600460u, 0x04600460u, 0x04600460u, 0x04600460u},
    {0x04800480u, 0x04800480u, 0x04800480u, 0x04800480u}, {0x04A004A0u, 0x04A004A0u, 0x04A004A0u, 0x04A004A0u},
    {0x04C004C0u, 0x04C004C0u, 0x04C004C0u, 0x04C004C0u}, {0x04E004E0u, 0x04E004E0u, 0x04E004E0u, 0x04E004E0u},
    {0x05000500u, 0x05000500u, 0x05000500u, 0x05000500u}, {0x05200520u, 0x05200520u, 0x05200520u, 0x05200520u},
    {0x05400540u, 0x05400540u, 0x05400540u, 0x05400540u}, {0x05600560u, 0x05600560u, 0x05600560u, 0x05600560u},
    {0x05800580u, 0x05800580u, 0x05800580u, 0x05800580u}, {0x05A005A0u, 0x05A005A0u, 0x05A005A0u, 0x05A005A0u},
    {0x05C005C0u, 0x05C005C0u, 0x05C005C0u, 0x05C005C0u}, {0x05E005E0u, 0x05E005E0u, 0x05E005E0u, 0x05E005E0u},
    {0x06000600u, 0x06000600u, 0x06000600u, 0x06000600u}, {0x06200620u, 0x06200620u, 0x06200620u, 0x06200620u},
    {0x06400640u, 0x06400640u, 0x06400640u, 0x06400640u}, {0x06600660u, 0x06600660u, 0x06600660u, 0x06600660u},
    {0x06800680u, 0x06800680u, 0x06800680u, 0x06800680u}, {0x06A006A0u, 0x06A006A0u, 0x06A006A0u, 0x06A006A0u},
    {0x06C006C0u, 0x06C006C0u, 0x06C006C0u, 0x06C006C0u}, {0x06E006E0u, 0x06E006E0u, 0x06E006E0u, 0x06E006E0u},
    {0x07000700u, 0x07000700u, 0x07000700u, 0x07000700u}, {0x07200720u, 0x07200720u, 0x07200720u, 0x07200720u},
    {0x07400740u, 0x07400740u, 0x07400740u, 0x07400740u}, {0x07600760u, 0x07600760u, 0x07600760u, 0x07600760u},
    {0x07800780u, 0x07800780u, 0x07800780u, 0x07800780u}, {0x07A007A0u, 0x07A007A0u, 0x07A007A0u, 0x07A007A0u},
    {0x07C007C0u, 0x07C007C0u, 0x07C007C0u, 0x07C007C0u}, {0x07E007E0u, 0x07E007E0u, 0x07E007E0u, 0x07E007E0u}};
constexpr int kSel = DPS_KSEL;

// The wave raises its issue priority while it computes and issues a batch of
// chunk loads and drops it after (s_setprio 1 / 0): the SIMD's arbiter then
// favours a wave that is about to put loads in flight over waves in their
// scatter or epilogue, so more loads overlap -- config3 k_cct1 66.2-66.3 ms
// against 67.1 ms at priority 0, the same output (profiles/r04/exp/ab_prio.txt;
// priority 3 the same as 1).
#ifndef DPS_PRIO_ISSUE
#define DPS_PRIO_ISSUE 1
#endif
__device__ __forceinline__ void issue1(const Stage& S, int b, const uint32_t* __restrict__ ent,
                                       int lane, Batch& B) {
#if DPS_PRIO_ISSUE
  __builtin_amdgcn_s_setprio(DPS_PRIO_ISSUE);
#endif
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const int q0 = b * (kWave * kU) + u * kWave;   // wave-uniform
    B.c[u] = 0;
    B.e[u] = make_uint4(0, 0, 0, 0);
    if (q0 >= S.G.nq) continue;
    const int q = q0 + lane;
    const bool live = q < S.G.nq;
    const int qlast = min(q0 + kWave - 1, S.G.nq - 1);
    const int jlo = __popcll(ballot(S.G.pre <= q0)) - 1;
    const int jhi = __popcll(ballot(S.G.pre <= qlast)) - 1;
    uint32_t bj = readlane(S.G.base, jlo);
    int cj = readlane(S.G.c, jlo);
    if (jhi > jlo) {
      if (jhi - jlo <= kSel) {
        for (int j = jlo + 1; j <= jhi; ++j) {   // wave-uniform loop
          const bool ge = q >= readlane(S.G.pre, j);
          const uint32_t bn = readlane(S.G.base, j);
          const int cn = readlane(S.G.c, j);
          bj = ge ? bn : bj;
          cj = ge ? cn : cj;
        }
      } else {
        int j = jlo;
        for (int jj = jlo + 1; jj <= jhi; ++jj) j += q >= readlane(S.G.pre, jj) ? 1 : 0;
        bj = static_cast<uint32_t>(__shfl(static_cast<int>(S.G.base), j, kWave));
        cj = __shfl(S.G.c, j, kWave);
      }
    }
    // (the offset wraps in 32 bits on purpose: base_j = lo_j - 4 pre_j may be
    // "negative", base_j + 4q is not)
    const uint32_t off = bj + 4u * static_cast<uint32_t>(q);
#ifdef DPS_DEBUG
    {
      // a live lane's chunk lies inside its own venue's bucket [lo_j, hi_j) =
      // [tile_off[b], tile_off[b+1]): its venue is the last lane j with
      // pre_j <= q (pre is nondecreasing; lanes past the group hold pre = nq).
      // Round 5's fault was this offset formed as pointer + a
      // "negative" 32-bit base before the positive 4q was added.
      int jt = -1;
      for (int j = 0; j < kWave; ++j) jt += readlane(S.G.pre, j) <= q ? 1 : 0;
      const int js = jt < 0 ? 0 : jt;
      const uint32_t base_j = static_cast<uint32_t>(__shfl(static_cast<int>(S.G.base), js, kWave));
      const int pre_j = __shfl(S.G.pre, js, kWave);
      const int pre_n = js + 1 < kWave ? __shfl(S.G.pre, js + 1, kWave) : S.G.nq;
      const uint32_t lo_j = base_j + 4u * static_cast<uint32_t>(pre_j);
      const uint32_t len_j = 4u * static_cast<uint32_t>(pre_n - pre_j);
      // (recorded, not trapped: counter[48..55] = line, q, off, bj, base_j,
      // pre_j, pre_n, nq of the first failing lane; tools/debug_checks.py)
      // (bitwise, not short-circuit: the bpermutes above must run on every
      // lane -- sunk into a branch over the live lanes, -O1 code read 0 from
      // the lanes it had switched off and recorded false failures)
      const bool ok_lane = (jt >= 0) & (bj == base_j) & (off - lo_j < len_j);
      const bool bad = live & !ok_lane;
      if (bad) {
        unsigned long long* ctr = kcold(counter);
        if (atomicCAS(ctr + 48, 0ull, static_cast<unsigned long long>(__LINE__)) == 0ull) {
          ctr[49] = static_cast<unsigned long long>(q);
          ctr[50] = off;
          ctr[51] = bj;
          ctr[52] = base_j;
          ctr[53] = static_cast<unsigned long long>(pre_j);
          ctr[54] = static_cast<unsigned long long>(pre_n);
          ctr[55] = static_cast<unsigned long long>(S.G.nq) | (static_cast<unsigned long long>(jt + 1) << 32);
        }
      }
    }
#endif
    const uint4* src = live ? reinterpret_cast<const uint4*>(ent + off) : kDeadChunk + lane;
    B.e[u] = *src;
    B.c[u] = live ? cj : 0;
  }
#if DPS_PRIO_ISSUE
  __builtin_amdgcn_s_setprio(0);
#endif
}

// Venues 64.. of a row with more than 64 venues: their buckets of tile t,
// loaded and scattered synchronously (pass `pass` of mode lnp).
template <int F, bool T15>
__device__ __forceinline__ int extra_groups(const CctParams& p, const Stage& S, uint32_t* acc,
                                            int64_t pb, int d, int lane, bool u8h) {
  const uint32_t* off = u8h ? p.h_off : p.tile_off;
  const uint32_t* ent = u8h ? p.h_ent : p.tile_ent;
  const uint32_t T = static_cast<uint32_t>(u8h ? p.T8 : p.T);
  int chunks = 0;
  for (int g0 = kWave; g0 < d; g0 += kWave) {
    const int j = g0 + lane;
    uint32_t lo = 0, hi = 0;
    int c = 0;
    if (j < d) {
      const uint32_t b = static_cast<uint32_t>(kcold(c_col)[pb + j]) * T + static_cast<uint32_t>(S.t);
      lo = off[b];
      hi = off[b + 1];
      c = kcold(c_val)[pb + j];
    }
    Stage E = S;
    grp_set(E.G, lo, hi, c, d - g0 < kWave ? d - g0 : kWave);
    E.nb = (E.G.nq + kWave * kU - 1) / (kWave * kU);
    chunks += E.G.nq;
    for (int b = 0; b < E.nb; ++b) {
      Batch B;
      issue1(E, b, ent, lane, B);
      scatter_f<F, T15>(B, E, b, acc, u8h);
    }
  }
  return chunks;
}

// Top-k lists up to DPS_W5_KPL * 64 slots run 5 waves per SIMD (96 VGPRs),
// longer ones 4 (128 VGPRs).
#ifndef DPS_W5_KPL
#define DPS_W5_KPL 1
#endif
// OPT: the optimistic 4-bit passes compiled in (launched only with tile_sum:
// the instantiation without them keeps the old register allocation -- the
// redo queue and the check alone cost 3 ms of the non-optimistic launch).
// kcold() reads CctParams fields from the kernarg segment at their offsetof:
// valid only while the by-value CctParams is k_cct1's FIRST and ONLY argument
// (kernarg offset 0) and only in code inlined into k_cct1 (win_ub,
// extra_groups and the row loop).  Do not add a kernel argument or call a
// kcold-using helper from another kernel.
static_assert(std::is_trivially_copyable<CctParams>::value, "CctParams is passed by value");
template <int F, int KPL, bool HV, bool SY, bool OPT, bool T15>
// The symmetric-mode instantiation carries the record path and the published
// bounds: DPS_SYM_WPE waves per SIMD (4: 128 VGPRs, no spills).
#ifndef DPS_SYM_WPE
#define DPS_SYM_WPE 4
#endif
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(
    SY ? DPS_SYM_WPE : KPL <= DPS_W5_KPL ? 5 : 4))) void k_cct1(CctParams p) {
  // LDS: the accumulator at address 0 (scatter ORs the in-tile offset into 0)
  // then the candidate queue.
  static_assert(!T15 || (!SY && !OPT), "the T15 layout has no symmetric or optimistic passes");
  __shared__ __attribute__((aligned(16))) uint32_t lds[Geo<F, T15>::ACC_DW];
  uint32_t* acc = lds;
  const int lane = lane_id();
  VQ Q;
  Q.lab0 = Q.m0 = Q.lab1 = Q.m1 = 0;
  Q.n = 0;
  for (int i = lane * 4; i < Geo<F, T15>::ACC_DW; i += kWave * 4)
    *reinterpret_cast<uint4*>(acc + i) = make_uint4(0, 0, 0, 0);
  // profiling aid (-DDPS_PROFILE build, DPATHSIM_ABLATE=16): shader-clock
  // cycles per phase (scatter, flush + thresholds, next-stage prefetch,
  // epilogue) and the stage count, summed over waves into counter[8..12]
  const bool prof = kProfile && (p.ablate & 16) != 0;
  // profiling build: this wave's realtime stamps (100 MHz, chip-wide), at
  // counter[64 + 4 * wave]: start, end, start of its last row, that row
  const uint64_t rt0 = prof ? __builtin_amdgcn_s_memrealtime() : 0;
  uint64_t rt_last = 0;
  int x_last = -1;
  uint64_t ts[7] = {0, 0, 0, 0, 0, 0, 0}, pc[7] = {0, 0, 0, 0, 0, 0, 0};
  // work counts of this wave (wave-uniform), summed into counter[1..2] at exit:
  // accumulator passes (each reads and zeroes the 8 KiB accumulator) and 16-byte
  // chunks scattered -- the bench's algorithmic LDS bytes
  uint32_t n_pass = 0, n_chunk = 0;   // < 2^32 per wave (widened at the exit)
  RowAux ra;       // work counts; the symmetric mode's row state

  for (;;) {
    unsigned long long rr = 0;
    if (lane == 0) rr = atomicAdd(kcold(counter), 1ull);
    const int r = __builtin_amdgcn_readfirstlane(static_cast<int>(rr));
    if (r >= kcold(n_rows)) break;
    const int32_t* row_order = kcold(row_order);
    const int x = row_order ? row_order[r] : static_cast<int>(kcold(row_begin) + r);   // < 2^31
    uint32_t np_row = 0;                // profiling build: passes before this row
    if (prof) {
      rt_last = __builtin_amdgcn_s_memrealtime();
      x_last = r;
      np_row = n_pass;
    }
    const bool is_piece = r < kcold(n_pieces);
    int t_beg = is_piece ? kcold(piece_t0)[r] : 0;
    int t_end = is_piece ? kcold(piece_t1)[r] : static_cast<int>(p.T);
    DPS_DASSERT(0 <= t_beg && t_beg <= t_end && t_end <= p.T);
    const int32_t* t_rank = kcold(t_rank);
    const int x_lab = t_rank ? t_rank[x] : static_cast<int>(x);   // labels < 2^31
    const int64_t* c_ptr = kcold(c_ptr);
    const int64_t pb = c_ptr[x];
    const int d = static_cast<int>(c_ptr[x + 1] - pb);
    const int64_t gx = kcold(g)[x];
    const float gxf = i64_f32(gx);
    TopK<KPL> top;
    top.init(kcold(k));
    ra.x = static_cast<int>(x);
    ra.far = INT_MAX;
    bool strong = false;                // sym rest pass: a partial list, no zero fill
    if (SY) {
      const int a = static_cast<int>(x_lab >> p.shift);
      if (p.sym == 1) {                 // band pass: the row's own tile +- band
        t_beg = max(t_beg, a - p.band);
        t_end = min(t_end, a + p.band + 1);
      } else {                          // rest pass
        ra.far = a + p.band + 1;
        strong = p.row_strong[x] != 0;
        if (strong) {                   // tiles above the band, its k-th as the floor
          const int64_t e = static_cast<int64_t>(x) * p.k + p.k - 1;
          top.set_floor(p.seed_score[e], p.seed_idx[e]);
          t_beg = max(t_beg, ra.far);
        }
      }
    }

    if (d > 0 && t_beg < t_end) {
      const int d0 = d < kWave ? d : kWave;
      int c = 0, v = 0;
      uint32_t vT = 0;
      if (lane < d0) {
        c = kcold(c_val)[pb + lane];
        v = kcold(c_col)[pb + lane];
        vT = static_cast<uint32_t>(v) * static_cast<uint32_t>(p.T);
      }
      if (d0 > 1) sort_venues<HV || F == 2>(p, d0, lane, c, vT, v);
      // dual (F = 2): wide tiles run as two u8 halves of the companion set
      const bool dual = F == 2 && p.h_ent != nullptr;
      const uint32_t vT8 = dual ? static_cast<uint32_t>(v) * static_cast<uint32_t>(p.T8) : 0u;
      Win1 w;
      int h_next = -1;            // the second half of a split wide tile, pending
      uint32_t h_ub = 0;
      // bound of a u8 half from the window (kHalfSat: 65535 or more -> the
      // 4-bit tile's own bound ub4, which also covers the half)
      auto half_ub = [&](uint32_t h, uint32_t ub4) -> uint32_t {
        return h >= kHalfSat ? ub4 : h;
      };
      // next stage: the pending half, else the next live tile -- when dual and
      // its 4-bit bound exceeds 15, an optimistic 4-bit pass (opt) or, above
      // kOptMax, its two u8 halves
      const bool opt_ok = OPT && !SY && kOptMax > 0 && dual && d <= kWave;
      // the u8 halves of an overflowed opt tile, queued (they run after the
      // prefetched next stage: tiles may be visited in any order)
      // (t8 << 8 | bound, bound <= kOptMax <= 255).  At most four: a check
      // runs after its stage's transition, when the next two stages are
      // already chosen -- each of those may push two more -- and from then on
      // choose() pops one per stage and a half never overflows.
      uint32_t rq[4] = {0, 0, 0, 0};
      int rq_n = 0;
      auto choose = [&](double tau, int& tn, uint32_t& ubn, bool& u8n, bool& optn, uint32_t& hbo) {
        u8n = false;
        optn = false;
        hbo = 0;
        if (h_next >= 0) {
          tn = h_next;
          ubn = h_ub;
          u8n = true;
          h_next = -1;
          return;
        }
        if (rq_n > 0) {           // u8 halves of an overflowed opt tile
          tn = static_cast<int>(rq[0] >> 8);
          ubn = rq[0] & 0xFFu;
          u8n = true;
          rq[0] = rq[1];
          rq[1] = rq[2];
          rq[2] = rq[3];
          --rq_n;
          return;
        }
        uint32_t hbn = 0;
        tn = next_tile<SY>(p, w, t_end, pb, d, c, vT, vT8, dual, lane, tau, gxf, ubn, hbn, ra.far);
        if (!dual || tn < 0 || ubn <= Fmt<F>::UB0) return;
        // (judged in the epilogue, a half's candidates wait in the queue: with
        // the list not yet full every count is one, so no opt pass then)
        if (opt_ok && ubn <= kOptMax && (!DPS_OPT_INEPI || tau > 0.0)) {
          optn = true;
          hbo = hbn;
          return;
        }
        const int ta = 2 * tn, tb = 2 * tn + 1;
        const uint32_t ua = half_ub(hbn & 0xFFFFu, ubn);
        const uint32_t ubb = tb < p.T8 ? half_ub(hbn >> 16, ubn) : 0u;
        u8n = true;
        if (ua == 0) {            // only the second half holds this row's entries
          tn = tb;
          ubn = ubb;
          return;
        }
        tn = ta;
        ubn = ua;
        if (ubb > 0) { h_next = tb; h_ub = ubb; }
      };
      // venue skipping: lane j < d0 holds venue j's heavy-table slot (-1: none)
      // and an upper bound of C[x,v] / s_v (s_v >= C[x,v] > 0)
      uint32_t hv = kHvNone;    // hv_pack(C[x,v] / s_v rounded up, slot)
      uint64_t hm = 0;          // H: venue lanes no longer scattered
      if (HV && lane < d0) {
        const int sl = kcold(hv_slot)[v];
        if (sl >= 0)
          hv = hv_pack(static_cast<float>(static_cast<double>(c) / static_cast<double>(kcold(s)[v])) *
                           (1.0f + 0x1p-20f), sl);
      }
      win_load<SY>(p, w, t_beg, t_beg, t_end, pb, d, c, vT, vT8, dual, lane, -1.0, gxf, ra.far);
      uint32_t ub_t = 0, hb_t = 0;
      int t0;
      bool u8n, optn;
      choose(-1.0, t0, ub_t, u8n, optn, hb_t);
      if (t0 >= 0) {
        Pend1 P;
        pend_load<F, HV, SY, T15>(p, P, t0, ub_t, u8n, d0, vT, vT8, lane, ra.far, optn, hb_t);
        Stage1 X;
        stage_make<F>(X, P, c, d0, 0ull, lane);
        bool hchg = false;        // H grew at the last stage boundary
        Batch B;
        issue1(X.S, 0, X.u8h ? p.h_ent : p.tile_ent, lane, B);
        int t1;
        choose(-1.0, t1, ub_t, u8n, optn, hb_t);
        pend_load<F, HV, SY, T15>(p, P, t1, ub_t, u8n, d0, vT, vT8, lane, ra.far, optn, hb_t);
        for (;;) {
          const int npass = 1 << X.S.lnp;
          bool more = false;
          for (X.S.pass = 0; X.S.pass < npass; ++X.S.pass) {
            if (prof) ts[0] = __builtin_amdgcn_s_memtime();
            const uint32_t* ent = X.u8h ? p.h_ent : p.tile_ent;
            if (X.S.pass > 0) issue1(X.S, 0, ent, lane, B);
            scatter_f<F, T15>(B, X.S, 0, acc, X.u8h);
            for (int b = 1; b < X.S.nb; ++b) {
              Batch B2;
              issue1(X.S, b, ent, lane, B2);
              scatter_f<F, T15>(B2, X.S, b, acc, X.u8h);
            }
            n_chunk += static_cast<uint32_t>(X.S.G.nq);
            ++n_pass;
            if (d > kWave)
              n_chunk += static_cast<uint32_t>(extra_groups<F, T15>(p, X.S, acc, pb, d, lane, X.u8h));
            if (prof) ts[1] = __builtin_amdgcn_s_memtime();
            // score what is queued while the list is filling or the queue is
            // half full (one memory round trip per 64 candidates)
            if (Q.n > 0 && (!top.full() || Q.n >= DPS_FLUSH_AT))
              vq_flush<KPL, HV, SY>(p, Q, top, Q.n < kWave ? Q.n : kWave, gx, lane, c, hv, hm, ra);
            const double tau = top.full() ? top.kth_s : -1.0;
            int mseg = 1;
            if (tau > 0.0) {
              if (HV && hm) {
                // two lower bounds of the M_Q a target needs, the larger wins:
                //  M_Q >= tau (gx + gs) / 2 - rho gs   (M_H <= rho g[y]; rounded
                //    down in fp32, every rounding to nearest, the factors keep it
                //    below the exact value), and
                //  M_Q >= mneed(tau, gx + gs) - ubh     (M_H <= ubh, integers)
                float rho = 0.0f;   // >= max_{h in H} C[x,h] / s_h
                for (uint64_t m = hm; m; m &= m - 1)
                  rho = fmaxf(rho, hv_ratio(readlane(hv, __builtin_ctzll(m))));
                const float gs = X.gsf;
                const float r = static_cast<float>(tau) * (gxf + gs) * (0.5f * (1.0f - 0x1p-19f)) -
                                rho * gs * (1.0f + 0x1p-17f);
                // (selects, not branches: r is per lane)
                const int m1c = static_cast<int>(ceilf(fminf(fmaxf(r, 1.0f), 2147483000.0f)));
                const int m1 = r >= 2147483000.0f ? INT32_MAX : m1c;
                const int m2 = mneed_lo32(static_cast<float>(tau), gxf + gs) - X.ubh;
                mseg = m1 > m2 ? m1 : m2;
              } else {
                const int mn = mneed_lo32(static_cast<float>(tau), gxf + X.gsf);
                mseg = mn > 1 ? mn : 1;
              }
            }
            if (SY && X.tbf < __builtin_inff()) {
              // symmetric rest pass, far tile: also every count that can reach the
              // segment's smallest tau_emit (pairs this row hands on)
              const int my = mneed_lo32(X.tbf, gxf + X.gsf);
              mseg = min(mseg, my > 1 ? my : 1);
            }
            const bool last = X.S.pass + 1 == npass;
            // a one-load stage: the sparse epilogue (DPS_SPARSE_LOADS, off), run
            // after the transition while B still holds this stage's chunks
            const bool sparse = kSparseLoads > 0 && !T15 && !SY && !(OPT && X.opt) && X.S.lnp == 0 &&
                                d <= kWave && X.S.G.nq <= kWave;
            Stage S = X.S;
            const bool u8S = F == 1 || X.u8h;   // this stage's counters: u8 format
            const bool S_u8h = X.u8h;
            const uint64_t hmS = hm;   // this stage's H (the update below is for the next)
            // optimistic 4-bit pass: did any count reach 16?  (then the
            // accumulator is cleared and the tile's two u8 halves run next)
            // optimistic 4-bit pass: judged after the transition below, so the
            // next stage's first chunks are in flight during the check
            // (S_hb != 0 for an opt stage: its bound exceeds 15, so one half's
            // bound is positive; S_exp: the two halves' expected sums, 16 bits each)
            const uint32_t S_hb = OPT && X.opt ? X.hb : 0u;
            const uint32_t S_exp = X.exp;
            if (prof) ts[2] = __builtin_amdgcn_s_memtime();
            if (last) {
              // next stage: its bounds were loaded one stage ago; put its first
              // chunks in flight, then load the bounds of the one after
              bool row_done = false;
              hchg = false;
              if (static_cast<float>(tau) > w.tau) {
                w.live &= win_pass(w, tau, gxf) | w.ykeep;
                w.tau = static_cast<float>(tau);
                if (HV) {
                  // H = the heavy venues with C[x,h] / s_h <= tau / 2 (hr is an
                  // upper bound of the ratio, th a lower bound of tau / 2); with
                  // every venue in H no target can reach tau
                  const float th = static_cast<float>(tau) * (0.5f * (1.0f - 0x1p-20f));
                  const uint64_t h2 = ballot(hv_ratio(hv) <= th);   // (kHvNone: false)
                  hchg = h2 != hm;
                  hm = h2;
                  row_done = d <= kWave && __popcll(hm) == d0;   // hm is within lanes < d0
                }
              }
              // (an overflowed opt tile's halves are queued behind the
              // prefetched P; when P ran out, one empty stage -- nothing
              // scattered, an all-zero accumulator -- lets them load)
              more = (P.t >= 0 || rq_n > 0) && !row_done;
              if (more && P.t >= 0) {
                stage_make<F>(X, P, c, d0, hm, lane);
              } else {
                X.S.G.nq = 0;
                X.S.nb = 0;
                X.S.lnp = 0;
                X.opt = false;
              }
              if (prof) ts[5] = __builtin_amdgcn_s_memtime();
              // (a sparse stage issues the next batch after its epilogue: B
              // still holds this stage's chunks)
              if (!sparse) issue1(X.S, 0, X.u8h ? p.h_ent : p.tile_ent, lane, B);
              if (prof) ts[6] = __builtin_amdgcn_s_memtime();
              int tn = -1;
              if (more) choose(tau, tn, ub_t, u8n, optn, hb_t);
              pend_load<F, HV, SY, T15>(p, P, tn, ub_t, u8n, d0, vT, vT8, lane, ra.far, optn, hb_t);
            }
            if (sparse) {
              epi1_sparse<KPL, HV, SY>(p, acc, top, Q, B.e[0], static_cast<int>(S.t), u8S, lane,
                                       x_lab, gx, mseg, c, hv, hmS, ra);
              issue1(X.S, 0, X.u8h ? p.h_ent : p.tile_ent, lane, B);
            }

            // which halves of an optimistic pass have a count that reached 16?
            // (the epilogue clears them without judging them; they run again
            // as their u8 half tiles, queued for a later stage)
            uint32_t bmask = 0xFFu, bad = 0u;
#if DPS_OPT_INEPI
            const uint32_t oexp = S_hb != 0u ? (S_exp == 0u ? 0xFFFFFFFFu : S_exp) : 0u;
#else
            const uint32_t oexp = 0u;
            if (S_hb != 0u) {
#ifdef DPS_EXP_NOCHECK
              bmask = 0xFFu;       // experiment only: wrong results when a count overflows
#elif defined(DPS_EXP_CHECKONLY)
              {                    // experiment only: the check runs, its result is ignored
                const uint32_t bm = opt_check(acc, S_exp, lane);
                asm volatile("" ::"s"(bm));
              }
#else
              bmask = opt_check(acc, S_exp, lane);
#endif
              bad = (bmask & 0x0Fu ? 0u : 1u) | (bmask & 0xF0u ? 0u : 2u);
            }
#endif
            if (prof) ts[3] = __builtin_amdgcn_s_memtime();
            if (sparse) {
              // (judged and cleared above)
            } else if (S.lnp == 0) {
              if (u8S)
                epi1_u8<KPL, HV, SY, T15>(p, acc, top, Q, static_cast<int>(S.t), lane, x_lab, gx, mseg, c, hv,
                                 hmS, ra);
              else
                epi1_u4<KPL, HV, SY, T15>(p, acc, top, Q, static_cast<int>(S.t), lane, x_lab, gx, mseg, c, hv,
                                 hmS, ra, bmask, oexp, bad);
            } else if (u8S) {
              epi1_wide<1, KPL, HV, SY, T15>(p, acc, top, Q, S, lane, x_lab, gx, mseg, c, hv, hmS, ra);
            } else {
              epi1_wide<F, KPL, HV, SY, T15>(p, acc, top, Q, S, lane, x_lab, gx, mseg, c, hv, hmS, ra);
            }
            if (OPT && bad) {
              // halves of an optimistic pass with a count that reached 16: run
              // again as their u8 half tiles, queued for a later stage (half
              // bounds <= the opt tile's bound <= kOptMax: never saturated)
              ++ra.redo;
              const int ta = 2 * static_cast<int>(S.t), tb = ta + 1;
              const uint32_t ua = (bad & 1u) ? S_hb & 0xFFFFu : 0u;
              const uint32_t ubb = (bad & 2u) && tb < p.T8 ? S_hb >> 16 : 0u;
              auto push = [&](int t8, uint32_t u) {
                DPS_DASSERT(rq_n < 4);   // the bound argued at rq's declaration
                const uint32_t e = (static_cast<uint32_t>(t8) << 8) | u;
                if (rq_n == 0) rq[0] = e;
                else if (rq_n == 1) rq[1] = e;
                else if (rq_n == 2) rq[2] = e;
                else rq[3] = e;
                ++rq_n;
              };
              if (ua) push(ta, ua);
              if (ubb) push(tb, ubb);
              // the row had no stage left: one empty stage picks the halves up
              if (rq_n > 0 && !more && X.S.G.nq == 0 && hm != ballot(lane < d0)) more = true;
            }
            // the queue holds counts that miss hmS: complete them before the
            // next stage's (larger) H applies
            if (HV && hchg)
              while (Q.n > 0)
                vq_flush<KPL, HV, SY>(p, Q, top, Q.n < kWave ? Q.n : kWave, gx, lane, c, hv, hmS, ra);
            if (prof) {
              ts[4] = __builtin_amdgcn_s_memtime();
#pragma unroll
              for (int i = 0; i < 4; ++i) pc[i] += ts[i + 1] - ts[i];
              ++pc[4];
              if (last) { pc[5] += ts[5] - ts[2]; pc[6] += ts[6] - ts[5]; }
              ra.u8h += S_u8h ? 1u : 0u;            // passes over a u8 half tile
              ra.wide += S.lnp > 0 ? 1u : 0u;       // passes with wider counters
              const int nq = S.G.nq;
              const int hb = nq == 0 ? 0 : nq <= 16 ? 1 : nq <= 64 ? 2 : nq <= 128 ? 3
                           : nq <= 192 ? 4 : nq <= 384 ? 5 : nq <= 768 ? 6 : 7;
#pragma unroll
              for (int i = 0; i < 8; ++i)
                if (i == hb) {
                  ++ra.nqh[i];
                  ra.nqc[i] += static_cast<uint32_t>(nq);
                  ra.nqe[i] += ts[4] - ts[3];
                }
            }
            if (last) break;
          }
          if (!more) break;
        }
      }
      while (Q.n > 0) vq_flush<KPL, HV, SY>(p, Q, top, Q.n < kWave ? Q.n : kWave, gx, lane, c, hv, hm, ra);
    }

    // ranked entries, then zero-score targets in reference order, then -1
    const int kk = kcold(k);
    const int64_t ro = (is_piece || kcold(out_by_slot)) ? r : x - kcold(row_begin);
    int32_t* oi = (is_piece ? kcold(piece_idx) : kcold(out_idx)) + ro * kk;
    int64_t* oc = (is_piece ? kcold(piece_cnt) : kcold(out_cnt)) + ro * kk;
    double* os = (is_piece ? kcold(piece_score) : kcold(out_score)) + ro * kk;
#pragma unroll
    for (int q = 0; q < KPL; ++q) {
      const int slot = q * kWave + lane;
      if (slot < top.filled) { oi[slot] = top.y[q]; oc[slot] = top.m[q]; os[slot] = top.s[q]; }
    }
    const int64_t avail = p.n_targets - 1;
    const int want = (is_piece || strong) ? top.filled : static_cast<int>(avail < kk ? avail : kk);
    int slot = top.filled;
    for (int64_t yb = 0; slot < want && yb < p.n_targets; yb += kWave) {
      const int64_t yc = yb + lane;
      bool ok = yc < p.n_targets && yc != x;
      for (int q = 0; q < KPL; ++q) {
        for (int l = 0; l < kWave; ++l) {
          if (q * kWave + l >= top.filled) break;
#ifdef DPS_DEBUG
          // (the readlane outside the short-circuit: under it the -O1 debug
          // build read lanes whose ranked entry had never been loaded)
          const int yl = readlane(top.y[q], l);
          ok = ok && yl != static_cast<int>(yc);
#else
          // (the same at -O3, where this form allocates better: 58.0 vs 58.8 ms
          // for the whole config3 launch, profiles/r06/f)
          ok = ok && (readlane(top.y[q], l) != static_cast<int>(yc));
#endif
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
    for (int s2 = want + lane; s2 < kk; s2 += kWave) {
      oi[s2] = -1;
      oc[s2] = 0;
      os[s2] = 0.0;
    }
    if (SY && p.sym == 2) sym_publish<KPL>(p, x_lab, strong, top, lane);
    // profiling build: per dequeue slot r, (realtime ticks << 32) | passes of
    // the row, at counter[64 + 4 * 16384 + r] (tools/row_times.py)
    if (prof && lane == 0 && r < (1 << 21))
      p.counter[64 + 4 * 16384 + r] = ((__builtin_amdgcn_s_memrealtime() - rt_last) << 32) |
                                      static_cast<unsigned long long>(n_pass - np_row);
  }
  if (lane == 0 && (n_pass | n_chunk)) {
    unsigned long long* ctr = kcold(counter);
    atomicAdd(ctr + 1, static_cast<unsigned long long>(n_pass));
    atomicAdd(ctr + 2, static_cast<unsigned long long>(n_chunk));
    if (HV && ra.ver) atomicAdd(ctr + 3, static_cast<unsigned long long>(ra.ver));
    if (ra.redo) atomicAdd(ctr + 4, static_cast<unsigned long long>(ra.redo));
  }
  if (prof && lane == 0 && blockIdx.x < 16384) {
    unsigned long long* wt = p.counter + 64 + 4 * static_cast<int64_t>(blockIdx.x);
    wt[0] = rt0;
    wt[1] = __builtin_amdgcn_s_memrealtime();
    wt[2] = rt_last;
    wt[3] = static_cast<unsigned long long>(static_cast<long long>(x_last));
  }
  if (prof && lane == 0) {
#pragma unroll
    for (int i = 0; i < 7; ++i) atomicAdd(p.counter + 8 + i, static_cast<unsigned long long>(pc[i]));
    atomicAdd(p.counter + 15, static_cast<unsigned long long>(ra.cand));
    atomicAdd(p.counter + 16, static_cast<unsigned long long>(ra.ins));
    atomicAdd(p.counter + 17, static_cast<unsigned long long>(ra.u8h));
    atomicAdd(p.counter + 18, static_cast<unsigned long long>(ra.wide));
#pragma unroll
    for (int i = 0; i < 5; ++i) atomicAdd(p.counter + 19 + i, static_cast<unsigned long long>(ra.bk[i]));
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      atomicAdd(p.counter + 24 + i, static_cast<unsigned long long>(ra.nqh[i]));
      atomicAdd(p.counter + 32 + i, static_cast<unsigned long long>(ra.nqc[i]));
      atomicAdd(p.counter + 40 + i, static_cast<unsigned long long>(ra.nqe[i]));
    }
  }
}

template <int F, int KPL, bool T15>
int launch1(const CctParams& p, hipStream_t st) {
  int dev = 0, n_cu = 256;
  DPS_HIP_RET(hipGetDevice(&dev));
  DPS_HIP_RET(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
  // 5 or 4 waves per SIMD by registers; the 8 KiB layout keeps 18 resident per
  // CU by LDS (Geo), the T15 layout 20 (a grid of 20 measured the same as 18
  // for 8 KiB: the two late workgroups per CU start at the end, profiles/r06/h)
  int wpc = KPL <= DPS_W5_KPL ? (T15 ? 20 : 18) : 16;
  if (p.sym) wpc = 4 * (DPS_SYM_WPE < (KPL <= DPS_W5_KPL ? 5 : 4) ? DPS_SYM_WPE : (KPL <= DPS_W5_KPL ? 5 : 4));
  if (const int t = tuning(DPS_TUNE_LEAN_WPC)) wpc = t;   // A/B of the occupancy
#ifdef DPS_PROFILE
  if (const char* e = std::getenv("DPATHSIM_LEAN_WPC")) wpc = std::atoi(e);   // experiments
  if (wpc < 1 || wpc > 20) wpc = 20;
#endif
  int64_t grid = static_cast<int64_t>(n_cu) * wpc;
  if (grid > p.n_rows) grid = p.n_rows;
  const auto g = static_cast<unsigned>(grid);
  if constexpr (T15) {        // (the caller rejects sym and tile_sum for this layout)
    if (p.hv_c) k_cct1<F, KPL, true, false, false, true><<<g, kWave, 0, st>>>(p);
    else k_cct1<F, KPL, false, false, false, true><<<g, kWave, 0, st>>>(p);
    DPS_LAUNCHED();
    return DPS_OK;
  }
  const bool opt = F == 2 && p.tile_sum != nullptr && p.h_ent != nullptr && kOptMax > 0;
  if (p.sym) k_cct1<F, KPL, false, true, false, false><<<g, kWave, 0, st>>>(p);
  else if (p.hv_c && opt) k_cct1<F, KPL, true, false, true, false><<<g, kWave, 0, st>>>(p);
  else if (p.hv_c) k_cct1<F, KPL, true, false, false, false><<<g, kWave, 0, st>>>(p);
  else if (opt) k_cct1<F, KPL, false, false, true, false><<<g, kWave, 0, st>>>(p);
  else k_cct1<F, KPL, false, false, false, false><<<g, kWave, 0, st>>>(p);
  DPS_LAUNCHED();
  return DPS_OK;
}

}  // namespace

// Lean kernel for W = 8192 (shift 13, u8 counters) and W = 16384 (shift 14,
// 4-bit counters), one wave per row; the caller has validated the parameters
// and zeroed p.counter.
int cct1_launch(const CctParams& p, hipStream_t st) {
  const bool t15 = p.tile_w != (1 << p.shift);
  if (p.shift == 13 && t15) {
    if (p.k <= 64) return launch1<1, 1, true>(p, st);
    if (p.k <= 128) return launch1<1, 2, true>(p, st);
    return launch1<1, 4, true>(p, st);
  }
  if (p.shift == 14 && t15) {
    if (p.k <= 64) return launch1<2, 1, true>(p, st);
    if (p.k <= 128) return launch1<2, 2, true>(p, st);
    return launch1<2, 4, true>(p, st);
  }
  if (p.shift == 13) {
    if (p.k <= 64) return launch1<1, 1, false>(p, st);
    if (p.k <= 128) return launch1<1, 2, false>(p, st);
    return launch1<1, 4, false>(p, st);
  }
  if (p.shift == 14) {
    if (p.k <= 64) return launch1<2, 1, false>(p, st);
    if (p.k <= 128) return launch1<2, 2, false>(p, st);
    return launch1<2, 4, false>(p, st);
  }
  return DPS_ERR_INVALID;
}

}  // namespace dps
