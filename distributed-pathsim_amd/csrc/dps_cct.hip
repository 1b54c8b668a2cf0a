// ★ Hot path: fused C.C^T + fp64 PathSim score + per-source top-k
// (replaces metapath_pairwise_walk
// DPathSim_APVPA.py:90-109, the score :51-52 and the target loop :18-22,36).
//
// Operands (see DESIGN.md "Data layout in HBM"):
//   C      CSR over author rows: int64 row_ptr, int32 col (venue), int32 val.
//   tiles  C^T cut into target tiles of W = 2^shift labels (targets relabeled
//          in ascending global walk g, dps_target_order).  Bucket (v,t) holds
//          packed entries -- W <= 8192: uint16 (l << 3) | e, l = label - t*W,
//          one power-of-two piece 2^e of C[y,v] (P16; e = 6, 7 at l % 4 == 3
//          are padding codes); wider: uint32 (C << 16) | (label - t*W) --
//          stored [v][t], each bucket padded to 16 bytes.
//   g_t    g in label order (ascending), tile_maxc max C per bucket.
//
// Default shape (W = 8192): one wave owns one source row at a time (persistent
// grid of single-wave workgroups, rows dequeued from an atomic counter,
// heaviest first); W >= 16384: 4 or 8 waves share a row.  For every target
// tile t in ascending g:
//   bound     UB = sum_v C[x,v] * maxc[v,t].  tau = the best k-th score held;
//             mneed = the smallest M whose score against the tile's smallest g
//             reaches tau.  UB < mneed: no target of the tile can enter the
//             top-k, skip it.
//   scatter   the row's buckets (v,t) are flattened into 16-byte chunks, 64
//             per load instruction; acc[y] += C[x,v]*c with no-return
//             ds_add_u32 into PACKED u8 accumulators (four targets per dword)
//             when UB <= 255, else u16 / u32 passes over parts of the tile.
//   epilogue  the accumulator is scanned (ds_read_b128) and zeroed in the same
//             pass; targets whose M reaches the threshold of their 1024-target
//             segment are queued and scored exactly: double(2M) / double(gx +
//             gy), one IEEE division, into the register top-k (lane i holds
//             rank i).
// At the row end the waves' lists are merged (one-wave rows write straight
// from registers), then the ranked entries, the zero-score fill (reference
// target order) and empty slots are written.
#include "dps_cct_dev.hpp"

#include <cstdlib>

namespace dps {
namespace {


// Bounds of the row's venues for tile tw (lane j = venue j, d <= 64): bucket
// (v_j, tw) is tile_ent[lo, hi), its largest C is mx.
struct Window {
  int64_t tw;
  int64_t tend;  // one past the last tile of this row (or row piece)
  int v, c;
  uint32_t vT;   // v * T: first bucket of venue v
  uint32_t lo, hi, mx;
  int64_t gmn;   // tile_gmin[tw], loaded one tile ahead
};

// Advance to the next tile that may hold a top-k target (d <= 64 rows).  The
// window's loads for the following tile are issued as soon as the current
// tile's values are consumed, so on a taken stage they complete behind the
// scatter and epilogue.
template <int NW>
__device__ __forceinline__ bool find_stage(const CctParams& p, Window& w, int d, int lane,
                                           float gxf, double tau_sh, int seg_shift,
                                           bool no_scatter, Stage& S) {
  const float tauf = static_cast<float>(tau_sh);
  while (w.tw < w.tend) {
    const int64_t t = w.tw++;
    const int64_t gmn = w.gmn;
    if (t + 1 < w.tend) w.gmn = p.tile_gmin[t + 1];
    const uint32_t lo = w.lo, hi = w.hi;
    // UB = sum_v C[x,v] * maxc[v,t] in 32 bits: a lane product of 2^25 or more
    // (or such a total) means "unbounded" -- no skip, 32-bit passes
    const uint64_t prod = static_cast<uint64_t>(static_cast<uint32_t>(w.c)) * w.mx;
    const uint32_t ub32 = wave_sum_u32(prod > (1u << 25) ? (1u << 25) : static_cast<uint32_t>(prod));
    int64_t ub = ub32 >= (1u << 25) ? (int64_t(1) << 40) : static_cast<int64_t>(ub32);
    w.lo = hi;
    if (lane < d && t + 1 < w.tend) {
      const uint32_t vb = w.vT + static_cast<uint32_t>(t) + 1u;   // < V*T + 1 < 2^32
      w.hi = p.tile_off[vb + 1];
      w.mx = p.tile_maxc[vb];
    }
    if (!p.use_bounds) ub = int64_t(1) << 40;
    const bool take = (kProfile && (p.ablate & 64))   // profiling aid: no bound test
                          ? true
                          : ub > 0 && (tau_sh <= 0.0 || ub >= mneed_lo32(tauf, gxf + i64_f32(gmn)));
    if ((kProfile && (p.ablate & 8)) && threadIdx.x == 0) {   // counters: tiles visited, tiles scanned
      atomicAdd(p.counter + 4, 1ull);
      if (take) atomicAdd(p.counter + 5, 1ull);
    }
    if (!take) continue;
    S.t = t;
    S.lnp = ub <= 0xFF ? 0 : ub <= 0xFFFF ? 1 : 2;
    S.pass = 0;
    grp_set(S.G, lo, hi, w.c, d);
    if (no_scatter) S.G.nq = 0;
    S.nb = (S.G.nq + NW * kWave * kU - 1) / (NW * kWave * kU);
    S.gq = p.g_t[min((t << p.shift) + (static_cast<int64_t>(lane) << seg_shift),
                     p.n_targets - 1)];
    return true;
  }
  S.G.base = 0; S.G.c = 0; S.G.pre = 0; S.G.nq = 0; S.G.nv = 1;   // no stage: dead loads only
  S.nb = 0;
  return false;
}

// Entry format of the tiles (dps_ct_tiles_build): P16 = 16-bit entries
// (W <= 8192), else 32-bit entries.
template <int KPL, int NW, bool P16>
__global__ __launch_bounds__(NW * kWave) __attribute__((amdgpu_waves_per_eu(4))) void k_cct_topk(CctParams p, int acc_dw) {
  // All LDS is dynamic, so the accumulators start at LDS address 0 and each
  // stage buffer is W-byte aligned (scatter_u8 ORs the in-tile offset in).
  // Layout: [2 stage buffers | per-wave queues | tau_s | fill_s | row_s].
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  double (*tau_s)[NW] = reinterpret_cast<double (*)[NW]>(lds + acc_dw + NW * 2 * kQ);
  int* fill_s = reinterpret_cast<int*>(lds + acc_dw + NW * 2 * kQ + 4 * NW);
  long long& row_s = *reinterpret_cast<long long*>(lds + acc_dw + NW * 2 * kQ + 5 * NW);
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_u32*)lds));
  const uint32_t lab_mask = ((1u << p.shift) - 1u) & ~3u;
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);   // wave-uniform (SGPR)
  const int nbuf = 1 << (p.shift - 2);        // accumulator dwords per stage buffer
  // threshold segments of min(1024, W/4) targets: one epilogue iteration each
  const int seg_shift = p.shift - 2 < 10 ? p.shift - 2 : 10;
  const bool no_add = kProfile && (p.ablate & 1) != 0;
  const bool no_scatter = kProfile && (p.ablate & 4) != 0;
  CandQ Q;
  Q.lab = reinterpret_cast<int*>(lds + acc_dw) + wave * 2 * kQ;
  Q.m = Q.lab + kQ;
  Q.n = 0;
  for (int i = tid; i < acc_dw; i += NW * kWave) lds[i] = 0;

  for (;;) {
    if (tid == 0) row_s = static_cast<long long>(atomicAdd(p.counter, 1ull));
    __syncthreads();
    const int64_t r = row_s;
    if (r >= p.n_rows) break;
    const int64_t x = p.row_order ? static_cast<int64_t>(p.row_order[r]) : p.row_begin + r;
    const bool is_piece = r < p.n_pieces;
    const int64_t ro = (is_piece || p.out_by_slot) ? r : x - p.row_begin;   // output row
    DPS_DASSERT(ro >= 0);
    // target tiles of this slot: the whole row, or one piece of a split row
    const int64_t t_beg = is_piece ? static_cast<int64_t>(p.piece_t0[r]) : 0;
    const int64_t t_end = is_piece ? static_cast<int64_t>(p.piece_t1[r]) : p.T;
    DPS_DASSERT(0 <= t_beg && t_beg <= t_end && t_end <= p.T);
    const int64_t x_lab = p.t_rank ? static_cast<int64_t>(p.t_rank[x]) : x;
    const int64_t pb = p.c_ptr[x];
    const int d = static_cast<int>(p.c_ptr[x + 1] - pb);
    DPS_DASSERT(d >= 0);
    const int64_t gx = p.g[x];
    const float gxf = i64_f32(gx);
    TopK<KPL> top;
    top.init(p.k);
    double tau_sh = -1.0;   // best k-th score of the workgroup, two stages old
    int n = 0;              // stages done in this row (selects buffer / tau slot)

    if (d > 0 && d <= kWave) {
      // ---- stages in ascending g.  The two accumulator buffers alternate, so
      // a wave that finished scanning stage n goes straight on to stage n+1's
      // loads and adds while the others still scan: one barrier per stage.
      Window w;
      w.tw = t_beg;
      w.tend = t_end;
      w.v = 0; w.c = 0;
      w.lo = w.hi = w.mx = 0;
      w.vT = 0;
      w.gmn = t_beg < t_end ? p.tile_gmin[t_beg] : 0;
      if (lane < d && t_beg < t_end) {
        w.v = p.c_col[pb + lane];
        w.c = p.c_val[pb + lane];
        w.vT = static_cast<uint32_t>(w.v) * static_cast<uint32_t>(p.T);
        const int64_t vb = w.vT + static_cast<uint32_t>(t_beg);
        w.lo = p.tile_off[vb];
        w.hi = p.tile_off[vb + 1];
        w.mx = p.tile_maxc[vb];
      }
      Stage cur;
      bool have = find_stage<NW>(p, w, d, lane, gxf, tau_sh, seg_shift, no_scatter, cur);
      // Batch 0 of the current stage is loaded one epilogue ahead.  It is issued
      // unconditionally (a missing stage loads dead chunks with C = 0) so B has
      // one definition in the loop and the register allocator need not copy it
      // -- a copy would wait on the loads at once and expose their latency.
      Batch B;
      if (!have) cur.G.nq = 0;
      issue<NW>(cur, 0, p.tile_ent, wave, lane, B, no_add, p.ablate, p.counter);
      // profiling aid (DPATHSIM_ABLATE & 16): shader-clock cycles per phase
      const bool prof = kProfile && (p.ablate & 16) != 0;
      uint64_t ts[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pc[7] = {0, 0, 0, 0, 0, 0, 0};
      while (have) {
        if (prof) ts[0] = __builtin_amdgcn_s_memtime();
        const int bi = p.dbuf ? (n & 1) : 0;
        uint32_t* acc = lds + bi * nbuf;
        const uint32_t buf = lds0 + static_cast<uint32_t>(bi * nbuf) * 4u;
        scatter_any<P16>(B, cur, acc, buf, lab_mask, p.shift);
        for (int b = 1; b < cur.nb; ++b) {
          Batch B2;
          issue<NW>(cur, b, p.tile_ent, wave, lane, B2, no_add, p.ablate, p.counter);
          scatter_any<P16>(B2, cur, acc, buf, lab_mask, p.shift);
        }
        if (prof) ts[1] = __builtin_amdgcn_s_memtime();
        // score what is queued while the wave's list is filling or the queue is
        // half full (one memory round trip per 64 candidates); done here, while
        // no prefetch is in flight, so its loads do not wait on the prefetch
        if (Q.n > 0 && (!top.full() || Q.n >= kWave / 2))
          flush<KPL>(p, Q, top, Q.n, gx, tau_sh, lane);
        // (one-wave rows too: skipping this LDS round trip measured 7 % slower)
        if (lane == 0) tau_s[n & 1][wave] = top.full() ? top.kth_s : -1.0;
        if (prof) ts[2] = __builtin_amdgcn_s_memtime();
#ifdef DPS_NOBAR1
        if constexpr (NW > 1) __syncthreads();   // one wave: its own LDS ops are in order
#else
        __syncthreads();
#endif
        if (prof) ts[3] = __builtin_amdgcn_s_memtime();
        double tm = tau_s[n & 1][0];
#pragma unroll
        for (int i = 1; i < NW; ++i) tm = tau_s[n & 1][i] > tm ? tau_s[n & 1][i] : tm;
        tau_sh = tm;
        const int mseg = stage_mseg(top, cur, gxf, tau_sh);
        // find the next stage and put its first loads in flight before this
        // stage's epilogue (pure LDS work unless the queue fills up)
        Stage nxt;
        bool have_n;
        if (cur.pass + 1 < (1 << cur.lnp)) { nxt = cur; ++nxt.pass; have_n = true; }
        else have_n = find_stage<NW>(p, w, d, lane, gxf, tau_sh, seg_shift, no_scatter, nxt);
        if (!have_n) nxt.G.nq = 0;
        if (prof) ts[4] = __builtin_amdgcn_s_memtime();
        issue<NW>(nxt, 0, p.tile_ent, wave, lane, B, no_add, p.ablate, p.counter);
        if (prof) ts[5] = __builtin_amdgcn_s_memtime();
        if (kProfile && (p.ablate & 32)) {   // profiling aid: zero the accumulator only
          for (int i = wave * (nbuf / NW) + lane * 4; i < (wave + 1) * (nbuf / NW); i += kWave * 4)
            *reinterpret_cast<uint4*>(acc + i) = make_uint4(0, 0, 0, 0);
        } else {
          epilogue<KPL, NW>(p, acc, top, Q, cur, wave, lane, nbuf, seg_shift, x_lab, gx, tau_sh,
                            mseg);
        }
        if (prof) ts[6] = __builtin_amdgcn_s_memtime();
#ifdef DPS_NOBAR2
        if constexpr (NW > 1)
#endif
        if (!p.dbuf) __syncthreads();   // one buffer: every wave has zeroed its quarter
        if (prof) {
          ts[7] = __builtin_amdgcn_s_memtime();
#pragma unroll
          for (int i = 0; i < 7; ++i) pc[i] += ts[i + 1] - ts[i];
        }
        ++n;
        cur = nxt;
        have = have_n;
      }
      if (prof && lane == 0) {   // scatter, flush, barrier 1, find, prefetch, epilogue, barrier 2
#pragma unroll
        for (int i = 0; i < 7; ++i) atomicAdd(p.counter + 8 + i, static_cast<unsigned long long>(pc[i]));
        atomicAdd(p.counter + 15, static_cast<unsigned long long>(n));
      }
    } else if (d > kWave) {
      // ---- rows with more than 64 venues: the same stages, synchronously
      for (int64_t t = t_beg; t < t_end; ++t) {
        int64_t ub = 0;
        for (int g0 = 0; g0 < d; g0 += kWave) {
          const int j = g0 + lane;
          if (j < d)
            ub += static_cast<int64_t>(p.c_val[pb + j]) *
                  p.tile_maxc[static_cast<int64_t>(p.c_col[pb + j]) * p.T + t];
        }
        ub = wave_sum(ub);
        if (!p.use_bounds) ub = int64_t(1) << 40;
        if (ub == 0) continue;
        if (tau_sh > 0.0 && ub < mneed_lo32(static_cast<float>(tau_sh), gxf + i64_f32(p.tile_gmin[t])))
          continue;
        Stage S;
        S.t = t;
        S.lnp = ub <= 0xFF ? 0 : ub <= 0xFFFF ? 1 : 2;
        S.gq = p.g_t[min((t << p.shift) + (static_cast<int64_t>(lane) << seg_shift),
                         p.n_targets - 1)];
        for (S.pass = 0; S.pass < (1 << S.lnp); ++S.pass) {
          const int bi = p.dbuf ? (n & 1) : 0;
          uint32_t* acc = lds + bi * nbuf;
          const uint32_t buf = lds0 + static_cast<uint32_t>(bi * nbuf) * 4u;
          for (int g0 = 0; !no_scatter && g0 < d; g0 += kWave) {
            const int j = g0 + lane;
            uint32_t lo = 0, hi = 0;
            int c = 0;
            if (j < d) {
              const int64_t bk = static_cast<int64_t>(p.c_col[pb + j]) * p.T + t;
              lo = p.tile_off[bk];
              hi = p.tile_off[bk + 1];
              c = p.c_val[pb + j];
            }
            grp_set(S.G, lo, hi, c, d - g0 < kWave ? d - g0 : kWave);
                    S.nb = (S.G.nq + NW * kWave * kU - 1) / (NW * kWave * kU);
            for (int b = 0; b < S.nb; ++b) {
              Batch B;
              issue<NW>(S, b, p.tile_ent, wave, lane, B, no_add);
              scatter_any<P16>(B, S, acc, buf, lab_mask, p.shift);
            }
          }
          if (Q.n > 0 && (!top.full() || Q.n >= kWave / 2))
            flush<KPL>(p, Q, top, Q.n, gx, tau_sh, lane);
          if (lane == 0) tau_s[n & 1][wave] = top.full() ? top.kth_s : -1.0;
          __syncthreads();
          double tm = tau_s[n & 1][0];
#pragma unroll
          for (int i = 1; i < NW; ++i) tm = tau_s[n & 1][i] > tm ? tau_s[n & 1][i] : tm;
          tau_sh = tm;
          epilogue<KPL, NW>(p, acc, top, Q, S, wave, lane, nbuf, seg_shift, x_lab, gx, tau_sh,
                        stage_mseg(top, S, gxf, tau_sh));
          if (!p.dbuf) __syncthreads();
          ++n;
        }
      }
    }
    if (Q.n > 0) flush<KPL>(p, Q, top, Q.n, gx, tau_sh, lane);
    __syncthreads();   // every wave has finished scanning (and zeroing) its last stage

    // ---- merge the wave lists (the accumulators are all zero; reuse) ---
    double* ms = reinterpret_cast<double*>(lds);          // [NW][k]
    int* my = reinterpret_cast<int*>(ms + NW * p.k);     // [NW][k]
    int* mm = my + NW * p.k;                              // [NW][k]
    if constexpr (NW > 1) {   // one-wave rows write straight from registers
#pragma unroll
      for (int q = 0; q < KPL; ++q) {
        const int slot = q * kWave + lane;
        if (slot < top.filled) {
          ms[wave * p.k + slot] = top.s[q];
          my[wave * p.k + slot] = top.y[q];
          mm[wave * p.k + slot] = top.m[q];
        }
      }
      if (lane == 0) fill_s[wave] = top.filled;
      __syncthreads();
    }
    if (wave == 0) {
      for (int w = 1; w < NW; ++w) {
        const int nf = fill_s[w];
        for (int i = 0; i < nf; ++i) {
          const double cs = ms[w * p.k + i];
          const int cy = my[w * p.k + i];
          if (!better(cs, cy, top.kth_s, top.kth_y)) break;   // lists are sorted
          top.insert(cs, cy, mm[w * p.k + i]);
        }
      }
      // ranked entries, then zero-score targets in reference order, then -1
      int32_t* oi = (is_piece ? p.piece_idx : p.out_idx) + ro * p.k;
      int64_t* oc = (is_piece ? p.piece_cnt : p.out_cnt) + ro * p.k;
      double* os = (is_piece ? p.piece_score : p.out_score) + ro * p.k;
#pragma unroll
      for (int q = 0; q < KPL; ++q) {
        const int slot = q * kWave + lane;
        if (slot < top.filled) { oi[slot] = top.y[q]; oc[slot] = top.m[q]; os[slot] = top.s[q]; }
      }
      const int64_t avail = p.n_targets - 1;
      const int want = is_piece ? top.filled : static_cast<int>(avail < p.k ? avail : p.k);
      int slot = top.filled;
      for (int64_t yb = 0; slot < want && yb < p.n_targets; yb += kWave) {
        const int64_t yc = yb + lane;
        bool ok = yc < p.n_targets && yc != x;
#pragma unroll
        for (int q = 0; q < KPL; ++q) {
          for (int l = 0; l < kWave; ++l) {
            if (q * kWave + l >= top.filled) break;
            // (a plain AND, not &&: see the same loop in dps_cct1.hip)
            const int yl = readlane(top.y[q], l);
            ok = ok & (yl != static_cast<int>(yc));
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
    if constexpr (NW > 1) {
      __syncthreads();
      for (int i = tid; i < NW * p.k * 4; i += NW * kWave) lds[i] = 0;   // 16 B per merge entry
    }
  }
}

// Split rows: one wave per row merges the ranked lists of its P pieces (each
// sorted by (score desc, y asc), -1 after its last entry) -- lane j holds the
// head of list j, a wave arg-best picks the next entry -- then fills zero-score
// targets in reference order and -1, exactly as the kernel's row end does.
constexpr int kMergeMaxK = 256;

__global__ __launch_bounds__(256) void k_topk_merge(
    const int32_t* __restrict__ p_idx, const int64_t* __restrict__ p_cnt,
    const double* __restrict__ p_score, const int32_t* __restrict__ rows, int64_t n_groups, int P,
    int k, int64_t n_targets, int64_t row_begin, int32_t* __restrict__ out_idx,
    int64_t* __restrict__ out_cnt, double* __restrict__ out_score) {
  __shared__ int32_t ranked_s[4][kMergeMaxK];
  const int lane = lane_id();
  const int wave = threadIdx.x / kWave;
  int32_t* ranked = ranked_s[wave];
  const int64_t wave0 = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) / kWave;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * (blockDim.x / kWave);
  for (int64_t grp = wave0; grp < n_groups; grp += nwaves) {
    const int64_t x = rows[grp * P];
    const int64_t ro = x - row_begin;
    int32_t* oi = out_idx + ro * k;
    int64_t* oc = out_cnt + ro * k;
    double* os = out_score + ro * k;
    const int64_t base = (grp * P + lane) * static_cast<int64_t>(k);   // list of lane j
    int h = 0;
    double hs = -1.0;
    int hy = INT_MAX;
    if (lane < P && p_idx[base] >= 0) { hs = p_score[base]; hy = p_idx[base]; }
    int filled = 0;
    for (; filled < k; ++filled) {
      // wave arg-best over the heads (score desc, then y asc)
      double bs = hs;
      int by = hy, bl = lane;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        const double os2 = __shfl_xor(bs, off, kWave);
        const int oy = __shfl_xor(by, off, kWave);
        const int ol = __shfl_xor(bl, off, kWave);
        if (better(os2, oy, bs, by)) { bs = os2; by = oy; bl = ol; }
      }
      if (by == INT_MAX) break;   // every list is exhausted
      if (lane == bl) {
        const int64_t e = base + h;
        oi[filled] = hy;
        oc[filled] = p_cnt[e];
        os[filled] = hs;
        ranked[filled] = hy;
        ++h;
        hs = -1.0;
        hy = INT_MAX;
        if (h < k && p_idx[base + h] >= 0) { hs = p_score[base + h]; hy = p_idx[base + h]; }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int64_t avail = n_targets - 1;
    const int want = static_cast<int>(avail < k ? avail : k);
    int slot = filled;
    for (int64_t yb = 0; slot < want && yb < n_targets; yb += kWave) {
      const int64_t yc = yb + lane;
      bool ok = yc < n_targets && yc != x;
      for (int q = 0; q < filled && ok; ++q) ok = ranked[q] != static_cast<int>(yc);
      const uint64_t mk = ballot(ok);
      const int rank = mbcnt(mk);
      if (ok && slot + rank < want) {
        oi[slot + rank] = static_cast<int32_t>(yc);
        oc[slot + rank] = 0;
        os[slot + rank] = 0.0;
      }
      slot += __popcll(mk);
    }
    for (int s2 = want + lane; s2 < k; s2 += kWave) {
      oi[s2] = -1;
      oc[s2] = 0;
      os[s2] = 0.0;
    }
    __builtin_amdgcn_wave_barrier();
  }
}

int log2_exact(int32_t w) {
  int s = 0;
  while (s < 31 && (1 << s) < w) ++s;
  return (1 << s) == w ? s : -1;
}

template <int KPL, int NW, bool P16>
int launch(const CctParams& p, hipStream_t st) {
  // one or two stage buffers of W/4 dwords; the row-end merge reuses them (16 B
  // per entry)
  int acc_dw = (p.dbuf ? 2 : 1) * (1 << (p.shift - 2));
  if (acc_dw < 4 * NW * p.k) acc_dw = 4 * NW * p.k;
  // + tau_s (2*NW doubles) + fill_s (NW ints) + row_s (one 8-byte slot)
  const size_t lds = (static_cast<size_t>(acc_dw) + NW * 2 * kQ + 5 * NW + 2) * sizeof(uint32_t);
  DPS_HIP_RET(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_cct_topk<KPL, NW, P16>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  static_cast<int>(lds)));
  int dev = 0, n_cu = 256;
  DPS_HIP_RET(hipGetDevice(&dev));
  DPS_HIP_RET(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
  int per_cu = static_cast<int>((160 * 1024) / (lds + 256));
  if (per_cu < 1) per_cu = 1;
  if (per_cu > 16 / NW) per_cu = 16 / NW;   // 4 waves per SIMD (128 VGPRs each)
  int64_t grid = static_cast<int64_t>(n_cu) * per_cu;
  if (grid > p.n_rows) grid = p.n_rows;
  k_cct_topk<KPL, NW, P16><<<static_cast<unsigned>(grid), NW * kWave, lds, st>>>(p, acc_dw);
  DPS_LAUNCHED();
  return DPS_OK;
}

template <bool P16>
int dispatch(const CctParams& p, int nw, int k, hipStream_t st) {
  if (nw == 8) {   // 64 KB of u8 accumulators: 8-wave workgroups, two per CU
    if constexpr (P16) {
      return DPS_ERR_INVALID;   // never: 8 waves only for W = 65536
    } else {
      if (k <= 64) return launch<1, 8, P16>(p, st);
      if (k <= 128) return launch<2, 8, P16>(p, st);
      return launch<4, 8, P16>(p, st);
    }
  }
  if (nw == 1) {   // one wave per row
    if (k <= 64) return launch<1, 1, P16>(p, st);
    if (k <= 128) return launch<2, 1, P16>(p, st);
    return launch<4, 1, P16>(p, st);
  }
  if (k <= 64) return launch<1, 4, P16>(p, st);
  if (k <= 128) return launch<2, 4, P16>(p, st);
  return launch<4, 4, P16>(p, st);
}

// ---- heavy-first dequeue list (dps_heavy_first) ---------------------------
// Descending key of a row's work on a log scale, four steps per octave: one
// 8-bit radix pass orders the rows heaviest first (stable: equal keys keep the
// row order) -- the hot kernel's dequeue order is a load-balance heuristic
// and any order gives identical results.
__global__ __launch_bounds__(256) void k_work_key(const int64_t* __restrict__ work, int64_t n,
                                                  uint64_t* __restrict__ key) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t w = work[i];
    uint32_t b = 0;
    if (w > 0) {
      const uint64_t u = static_cast<uint64_t>(w);
      const int e = 63 - __clzll(static_cast<long long>(u));
      const uint32_t frac = static_cast<uint32_t>((u << (63 - e)) >> 61) & 3u;   // 2 bits below the top one
      b = 1u + 4u * static_cast<uint32_t>(e) + frac;                                 // <= 252
    }
    key[i] = 255u - b;
  }
}

// dq = the sorted rows (+ row_begin), the first n_split of them repeated
// `pieces` times in front (their piece slots), then the rest.
__global__ __launch_bounds__(256) void k_dequeue_list(const uint32_t* __restrict__ sorted, int64_t n,
                                                      int64_t row_begin, int64_t n_split,
                                                      int pieces, int32_t* __restrict__ dq) {
  const int64_t n_out = n + n_split * (pieces - 1);
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n_out;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t src = i < n_split * pieces ? i / pieces : i - n_split * (pieces - 1);
    dq[i] = static_cast<int32_t>(row_begin + sorted[src]);
  }
}

// ---- symmetric mode (dps_cct_sym) ------------------------------
// After the band pass (sym = 1): a row is "strong" when its band list holds k
// positive scores; its k-th score, rounded down to fp32, is the threshold other
// rows hand pairs on at (tau_emit, by target label; +inf: the row scans every
// tile itself and takes no records), tau_blk the minimum over 2048 labels,
// tau_tile over a tile.  (The rest pass runs in descending label order,
// k_desc_order, not heavy-first: a row's far targets have then mostly
// published their own k-th scores.)
__global__ __launch_bounds__(256) void k_sym_plan(
    int64_t n, int k, int shift, const int32_t* __restrict__ t_rank,
    const double* __restrict__ band_score, uint8_t* __restrict__ strong,
    float* __restrict__ tau_emit, uint32_t* __restrict__ tau_blk, uint32_t* __restrict__ tau_tile) {
  for (int64_t x = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; x < n;
       x += static_cast<int64_t>(gridDim.x) * 256) {
    const double kth = band_score[x * k + k - 1];
    const bool st = kth > 0.0;
    const int64_t lx = t_rank ? t_rank[x] : x;
    strong[x] = st ? 1 : 0;
    const float te = st ? __double2float_rd(kth) : __builtin_inff();
    tau_emit[lx] = te;
    if (st) {                                    // positive floats order as uints
      atomicMin(&tau_blk[lx >> 11], __float_as_uint(te));
      atomicMin(&tau_tile[lx >> shift], __float_as_uint(te));
    }
  }
}

__global__ __launch_bounds__(256) void k_desc_order(const int32_t* __restrict__ t_perm, int64_t n,
                                                    int32_t* __restrict__ dq) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * 256)
    dq[i] = t_perm ? t_perm[n - 1 - i] : static_cast<int32_t>(n - 1 - i);
}

// Records (y <- x, M) grouped by y: counts, then placement.
__global__ __launch_bounds__(256) void k_rec_count(const int32_t* __restrict__ rec_y,
                                                   const unsigned long long* __restrict__ rec_n,
                                                   int64_t cap, uint32_t* __restrict__ cnt) {
  const int64_t n = static_cast<int64_t>(*rec_n < static_cast<unsigned long long>(cap) ? *rec_n : cap);
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * 256)
    atomicAdd(&cnt[rec_y[i]], 1u);
}
__global__ __launch_bounds__(256) void k_rec_place(const int32_t* __restrict__ rec_y,
                                                   const int32_t* __restrict__ rec_x,
                                                   const int32_t* __restrict__ rec_m,
                                                   const unsigned long long* __restrict__ rec_n,
                                                   int64_t cap, const int64_t* __restrict__ off,
                                                   uint32_t* __restrict__ cur, int32_t* __restrict__ sx,
                                                   int32_t* __restrict__ sm) {
  const int64_t n = static_cast<int64_t>(*rec_n < static_cast<unsigned long long>(cap) ? *rec_n : cap);
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const int32_t y = rec_y[i];
    const int64_t pos = off[y] + atomicAdd(&cur[y], 1u);
    sx[pos] = rec_x[i];
    sm[pos] = rec_m[i];
  }
}

// Final lists, one wave per row: weak rows take their rest-pass list (a full
// scan, zero fill included); strong rows merge their band list (k positive
// entries, in out_*) with their rest-pass entries (those that beat its k-th)
// and their records (score recomputed exactly as the hot kernel does).
template <int KPL>
__global__ __launch_bounds__(256) void k_sym_merge(
    int64_t n, int k, const uint8_t* __restrict__ strong, const int64_t* __restrict__ den,
    const int32_t* __restrict__ r_idx, const int64_t* __restrict__ r_cnt,
    const double* __restrict__ r_score, const int64_t* __restrict__ off,
    const int32_t* __restrict__ sx, const int32_t* __restrict__ sm, int32_t* __restrict__ out_idx,
    int64_t* __restrict__ out_cnt, double* __restrict__ out_score) {
  const int lane = lane_id();
  const int64_t wave0 = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) / kWave;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * (blockDim.x / kWave);
  for (int64_t x = wave0; x < n; x += nwaves) {
    const int64_t base = x * k;
    if (!strong[x]) {
      for (int i = lane; i < k; i += kWave) {
        out_idx[base + i] = r_idx[base + i];
        out_cnt[base + i] = r_cnt[base + i];
        out_score[base + i] = r_score[base + i];
      }
      continue;
    }
    const int64_t rb = off[x], re = off[x + 1];
    const bool rest = r_idx[base] >= 0;
    if (!rest && rb == re) continue;             // the band list is the answer
    TopK<KPL> top;
    top.init(k);
#pragma unroll
    for (int r = 0; r < KPL; ++r) {
      const int slot = r * kWave + lane;
      if (slot < k) { top.s[r] = out_score[base + slot]; top.y[r] = out_idx[base + slot];
                      top.m[r] = static_cast<int>(out_cnt[base + slot]); }
    }
    top.filled = k;
    {
      const int rk = (k - 1) / kWave, lk = (k - 1) % kWave;
#pragma unroll
      for (int r = 0; r < KPL; ++r)
        if (r == rk) { top.kth_s = readlane(top.s[r], lk); top.kth_y = readlane(top.y[r], lk); }
    }
    const int64_t dx = den[x];
    const int64_t nr = rest ? k : 0;             // rest entries end at the first -1
    for (int64_t c0 = 0; c0 < nr + (re - rb); c0 += kWave) {
      const int64_t i = c0 + lane;
      bool cand = false;
      double sc = 0.0;
      int cy = 0, cm = 0;
      if (i < nr) {
        cy = r_idx[base + i];
        if (cy >= 0) { sc = r_score[base + i]; cm = static_cast<int>(r_cnt[base + i]); cand = true; }
      } else if (i < nr + (re - rb)) {
        const int64_t j = rb + (i - nr);
        cy = sx[j];
        cm = sm[j];
        sc = static_cast<double>(2 * static_cast<int64_t>(cm)) / static_cast<double>(dx + den[cy]);
        cand = true;
      }
      cand = cand && better(sc, cy, top.kth_s, top.kth_y);
      uint64_t mask = ballot(cand);
      while (mask) {
        const int srcl = __ffsll(static_cast<long long>(mask)) - 1;
        mask &= mask - 1;
        const double cs = readlane(sc, srcl);
        const int y = readlane(cy, srcl);
        if (!better(cs, y, top.kth_s, top.kth_y)) continue;
        top.insert(cs, y, readlane(cm, srcl));
      }
    }
#pragma unroll
    for (int r = 0; r < KPL; ++r) {
      const int slot = r * kWave + lane;
      if (slot < k) { out_idx[base + slot] = top.y[r]; out_cnt[base + slot] = top.m[r];
                      out_score[base + slot] = top.s[r]; }
    }
  }
}

// Band-pass work counts added into the rest pass's (kernel_counts reports both).
__global__ void k_add_counts(const unsigned long long* __restrict__ a, unsigned long long* __restrict__ b) {
  if (threadIdx.x >= 1 && threadIdx.x < 4) b[threadIdx.x] += a[threadIdx.x];
}

}  // namespace
}  // namespace dps


using namespace dps;

extern "C" {

// 64 counters; the profiling build adds four words per wave of the lean
// kernel (start, end, start of its last row, that row) for tools/wave_times.py
// (profiling build: + per-wave realtime stamps, 32 B x 16384 waves, and per-row
// time and passes, 8 B x 2^21 dequeue slots)
size_t dps_cct_topk_workspace_size(void) { return kProfile ? 512 + 32 * 16384 + 8 * (1 << 21) : 512; }

size_t dps_heavy_first_workspace_size(int64_t n_rows) {
  const size_t m = static_cast<size_t>(n_rows > 0 ? n_rows : 1);
  return 2 * align_up(m * sizeof(uint64_t)) + align_up(m * sizeof(uint32_t)) +
         align_up(radix_sort_workspace_size(n_rows)) + 1024;
}

int dps_heavy_first(const int64_t* work, int64_t n_rows, int64_t row_begin, int64_t n_split,
                    int32_t pieces, int32_t* dq, void* ws, size_t ws_bytes, void* stream) {
  DPS_REQUIRE(n_rows >= 0 && n_split >= 0 && n_split <= n_rows, DPS_ERR_INVALID,
              "need 0 <= n_split <= n_rows");
  DPS_REQUIRE(pieces >= 1 && pieces <= 64, DPS_ERR_INVALID, "pieces must be in [1, 64]");
  DPS_REQUIRE(row_begin >= 0 && row_begin + n_rows <= INT32_MAX, DPS_ERR_OVERFLOW,
              "row indices exceed int32");
  DPS_REQUIRE(reinterpret_cast<uintptr_t>(ws) % 256 == 0, DPS_ERR_WORKSPACE,
              "workspace not 256-byte aligned");
  DPS_REQUIRE(ws_bytes >= dps_heavy_first_workspace_size(n_rows), DPS_ERR_WORKSPACE,
              "heavy_first workspace too small");
  if (n_rows == 0) return DPS_OK;
  DPS_REQUIRE(work && dq, DPS_ERR_INVALID, "null work / dq");
  auto st = static_cast<hipStream_t>(stream);
  Carve c(ws, ws_bytes);
  uint64_t* key = c.take<uint64_t>(n_rows);
  uint64_t* key_sorted = c.take<uint64_t>(n_rows);
  uint32_t* rows = c.take<uint32_t>(n_rows);
  const size_t rws_bytes = radix_sort_workspace_size(n_rows);
  void* rws = c.take<char>(rws_bytes);
  DPS_REQUIRE(c.ok, DPS_ERR_WORKSPACE, "heavy_first workspace carve failed");
  k_work_key<<<grid_for(n_rows, 256), 256, 0, st>>>(work, n_rows, key);
  DPS_LAUNCHED();
  DPS_HIP_RET(radix_sort_pairs(key, nullptr, key_sorted, rows, n_rows, 8, rws, rws_bytes, st));
  const int64_t n_out = n_rows + n_split * (pieces - 1);
  k_dequeue_list<<<grid_for(n_out, 256), 256, 0, st>>>(rows, n_rows, row_begin, n_split, pieces, dq);
  DPS_LAUNCHED();
  return DPS_OK;
}

// Symmetric-mode state of one hot-kernel launch (see CctParams).
struct SymSetup {
  int sym, band;
  const uint8_t* row_strong;
  const int32_t* seed_idx;
  const double* seed_score;
  float* tau_emit;
  float* tau_blk;
  float* tau_tile;
  uint32_t* blk_done;
  uint32_t* tile_done;
  int32_t *rec_y, *rec_x, *rec_m;
  unsigned long long* rec_n;
  int64_t rec_cap;
};

static int cct_topk_impl(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                         const int64_t* g, const int64_t* g_t, const int32_t* t_perm,
                         const int32_t* t_rank, int64_t n_targets, int64_t n_mids,
                         int32_t tile_w, const uint32_t* tile_off, const uint32_t* tile_ent,
                         const uint32_t* tile_maxc, const int64_t* tile_gmin,
                         const dps_cct_ext* ext, int64_t row_begin,
                         int64_t n_rows, const int32_t* row_order, bool out_by_slot, int32_t k,
                         int32_t* out_idx, int64_t* out_cnt, double* out_score, void* ws,
                         size_t ws_bytes, void* stream, int64_t n_pieces = 0,
                         const int32_t* piece_t0 = nullptr, const int32_t* piece_t1 = nullptr,
                         int32_t* piece_idx = nullptr, int64_t* piece_cnt = nullptr,
                         double* piece_score = nullptr, const SymSetup* sy = nullptr) {
  const TileDim td = tile_dim(tile_w);
  const int shift = td.shift;
  DPS_REQUIRE(shift >= 8 && shift <= 16, DPS_ERR_UNSUPPORTED,
              "tile_w must be a power of two in [256, 65536], 7680 or 15360, got %d", tile_w);
  DPS_REQUIRE(k >= 1 && k <= 256, DPS_ERR_UNSUPPORTED, "k must be in [1, 256], got %d", k);
  DPS_REQUIRE(n_targets < INT32_MAX, DPS_ERR_OVERFLOW, "n_targets exceeds int32");
  DPS_REQUIRE(n_mids * ((n_targets + tile_w - 1) / tile_w) < int64_t(UINT32_MAX), DPS_ERR_OVERFLOW,
              "n_mids * tiles exceeds the 32-bit bucket index");
  DPS_REQUIRE(!t_perm == !t_rank, DPS_ERR_INVALID, "t_perm and t_rank go together");
  DPS_REQUIRE(tile_gmin && g && tile_off && tile_ent, DPS_ERR_INVALID,
              "g, tile_off, tile_ent and tile_gmin are required");
  DPS_REQUIRE(ws && ws_bytes >= dps_cct_topk_workspace_size(), DPS_ERR_WORKSPACE,
              "cct_topk workspace too small");
  const bool vskip = ext && ext->s;
  if (vskip) {
    DPS_REQUIRE(ext->hv_slot && ext->hv_c, DPS_ERR_INVALID,
                "dps_cct_ext venue skipping needs s, hv_slot and hv_c");
    DPS_REQUIRE(ext->n_hv >= 1 && ext->n_hv <= 64, DPS_ERR_INVALID,
                "dps_cct_ext.n_hv must be in [1, 64], got %d", ext->n_hv);
  }
  const bool half = ext && ext->half_ent;
  if (half) {
    DPS_REQUIRE(shift == 14, DPS_ERR_INVALID, "companion u8 tiles need tile_w 16384 or 15360");
    DPS_REQUIRE(ext->half_off && (ext->half_maxc || !tile_maxc), DPS_ERR_INVALID,
                "dps_cct_ext companion tiles need half_off (and half_maxc with tile_maxc)");
  }
  auto st = static_cast<hipStream_t>(stream);
  if (n_rows == 0) return DPS_OK;
  CctParams p;
  p.s = vskip ? ext->s : nullptr;
  p.hv_slot = vskip ? ext->hv_slot : nullptr;
  p.hv_c = vskip ? ext->hv_c : nullptr;
  p.n_hv = vskip ? ext->n_hv : 0;
  p.h_off = half ? ext->half_off : nullptr;
  p.h_ent = half ? ext->half_ent : nullptr;
  p.h_maxc = half ? (tile_maxc ? ext->half_maxc : ext->half_off) : nullptr;
  p.T8 = (n_targets + tile_w / 2 - 1) / (tile_w / 2);   // companion half tiles
  p.tile_sum = half ? ext->tile_sum : nullptr;
  p.c_ptr = c_ptr; p.c_col = c_col; p.c_val = c_val;
  p.g = g; p.g_t = g_t ? g_t : g; p.t_perm = t_perm; p.t_rank = t_rank;
  p.tile_off = tile_off; p.tile_ent = tile_ent; p.tile_gmin = tile_gmin;
  p.tile_maxc = tile_maxc ? tile_maxc : tile_off;
  p.use_bounds = tile_maxc != nullptr;
  p.n_targets = n_targets;
  p.T = (n_targets + tile_w - 1) / tile_w;
  p.shift = shift;
  p.tile_w = tile_w;
  // waves per row: one wave owns a row for W <= 8192 (8 KB of u8 accumulators,
  // no barriers, one exact running top-k per row); wider tiles share a row
  // between the waves of a workgroup (4 x 32 KB or 2 x 64 KB per CU)
  // (W = 16384 holds 4-bit-counter entries, which only the lean kernel reads)
  int nw = shift <= 14 ? 1 : shift == 16 ? 8 : 4;
  if (const int t = tuning(DPS_TUNE_WAVES_PER_ROW)) nw = t;
#ifdef DPS_PROFILE
  if (const char* e = std::getenv("DPATHSIM_NW")) nw = std::atoi(e);   // experiments
#endif
  DPS_REQUIRE(nw == 1 || nw == 4 || nw == 8, DPS_ERR_INVALID, "waves per row must be 1, 4 or 8");
  DPS_REQUIRE(nw != 8 || shift > 14, DPS_ERR_INVALID, "8 waves per row need tile_w >= 32768");
  DPS_REQUIRE(nw == 1 || shift != 14, DPS_ERR_UNSUPPORTED,
              "tile_w 16384 (4-bit counter entries) runs one wave per row");
  DPS_REQUIRE(!td.t15 || (nw == 1 && !sy && !(half && ext->tile_sum)), DPS_ERR_UNSUPPORTED,
              "tile_w %d runs the one-wave kernel without the symmetric mode or the "
              "optimistic passes", tile_w);

  p.dbuf = nw > 1 && shift <= 14;   // 2 x W bytes of u8 accumulators up to W = 16384, one 32 KB buffer above
  p.row_begin = row_begin; p.row_order = row_order; p.out_by_slot = out_by_slot;
  p.n_pieces = n_pieces; p.piece_t0 = piece_t0; p.piece_t1 = piece_t1;
  p.piece_idx = piece_idx; p.piece_cnt = piece_cnt; p.piece_score = piece_score;
  p.n_rows = n_rows; p.k = k;
  p.out_idx = out_idx; p.out_cnt = out_cnt; p.out_score = out_score;
  p.counter = static_cast<unsigned long long*>(ws);
  p.ablate = 0;
  p.sym = 0;
  p.band = 0;
  p.row_strong = nullptr;
  p.seed_idx = nullptr;
  p.seed_score = nullptr;
  p.tau_emit = p.tau_blk = p.tau_tile = nullptr;
  p.blk_done = p.tile_done = nullptr;
  p.rec_y = p.rec_x = p.rec_m = nullptr;
  p.rec_n = nullptr;
  p.rec_cap = 0;
  if (sy) {
    DPS_REQUIRE((shift == 13 || shift == 14) && nw == 1 && !vskip && n_pieces == 0,
                DPS_ERR_UNSUPPORTED,
                "symmetric mode runs the one-wave kernel (tile_w 8192 / 16384), no venue "
                "skipping, no split rows");
    p.sym = sy->sym; p.band = sy->band; p.row_strong = sy->row_strong;
    p.seed_idx = sy->seed_idx; p.seed_score = sy->seed_score;
    p.tau_emit = sy->tau_emit; p.tau_blk = sy->tau_blk; p.tau_tile = sy->tau_tile;
    p.blk_done = sy->blk_done; p.tile_done = sy->tile_done;
    p.rec_y = sy->rec_y; p.rec_x = sy->rec_x; p.rec_m = sy->rec_m;
    p.rec_n = sy->rec_n; p.rec_cap = sy->rec_cap;
  }
  // Profiling aid only: the production build ignores DPATHSIM_ABLATE (an
  // ablated run returns wrong top-k lists), the -DDPS_PROFILE build honours it.
  if (kProfile)
    if (const char* ab = std::getenv("DPATHSIM_ABLATE")) p.ablate = std::atoi(ab);
  // word 0: row dequeue counter; words 1-3: the lean kernel's pass / chunk /
  // table-completed candidate counts, word 4 its overflowed optimistic passes
  // (the debug build also zeroes its check record, words 48..55)
  DPS_HIP_RET(hipMemsetAsync(p.counter, 0, (kDebug || (p.ablate & 24)) ? 512 : 8 * sizeof(unsigned long long), st));
  // the bench shape (W = 8192, one wave per row) runs the lean kernel
  // (dps_cct1.hip); DPATHSIM_LEAN=0 selects this file's general kernel
  bool lean = (shift == 13 || shift == 14) && nw == 1 && (p.ablate == 0 || p.ablate == 16);
#ifdef DPS_PROFILE
  if (const char* e = std::getenv("DPATHSIM_LEAN")) lean = lean && std::atoi(e) != 0;   // experiments
#endif
  if (lean || shift == 14 || td.t15) return cct1_launch(p, st);
  if (shift <= 13) return dispatch<true>(p, nw, k, st);   // 16-bit tile entries
  return dispatch<false>(p, nw, k, st);
}

int dps_cct_topk(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                 const int64_t* g, const int64_t* g_t, const int32_t* t_perm,
                 const int32_t* t_rank, int64_t n_targets, int64_t n_mids, int32_t tile_w,
                 const uint32_t* tile_off, const uint32_t* tile_ent, const uint32_t* tile_maxc,
                 const int64_t* tile_gmin, const dps_cct_ext* ext, int64_t row_begin,
                 int64_t row_end, const int32_t* row_order, int32_t k,
                 int32_t* out_idx, int64_t* out_cnt, double* out_score, void* ws,
                 size_t ws_bytes, void* stream) {
  DPS_REQUIRE(0 <= row_begin && row_begin <= row_end && row_end <= n_targets, DPS_ERR_INVALID,
              "row range [%lld, %lld) outside [0, %lld)", static_cast<long long>(row_begin),
              static_cast<long long>(row_end), static_cast<long long>(n_targets));
  return cct_topk_impl(c_ptr, c_col, c_val, g, g_t, t_perm, t_rank, n_targets, n_mids, tile_w,
                       tile_off, tile_ent, tile_maxc, tile_gmin, ext, row_begin,
                       row_end - row_begin, row_order, false, k, out_idx, out_cnt, out_score, ws, ws_bytes, stream);
}

int dps_cct_topk_rows(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                      const int64_t* g, const int64_t* g_t, const int32_t* t_perm,
                      const int32_t* t_rank, int64_t n_targets, int64_t n_mids, int32_t tile_w,
                      const uint32_t* tile_off, const uint32_t* tile_ent,
                      const uint32_t* tile_maxc, const int64_t* tile_gmin,
                      const dps_cct_ext* ext, const int32_t* rows,
                      int64_t n_rows, int32_t k, int32_t* out_idx, int64_t* out_cnt,
                      double* out_score, void* ws, size_t ws_bytes, void* stream) {
  DPS_REQUIRE(n_rows >= 0 && n_rows <= n_targets, DPS_ERR_INVALID, "bad n_rows %lld",
              static_cast<long long>(n_rows));
  DPS_REQUIRE(n_rows == 0 || rows, DPS_ERR_INVALID, "rows is required");
  return cct_topk_impl(c_ptr, c_col, c_val, g, g_t, t_perm, t_rank, n_targets, n_mids, tile_w,
                       tile_off, tile_ent, tile_maxc, tile_gmin, ext, 0, n_rows, rows, true, k,
                       out_idx, out_cnt, out_score, ws, ws_bytes, stream);
}

int dps_cct_topk_split(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                       const int64_t* g, const int64_t* g_t, const int32_t* t_perm,
                       const int32_t* t_rank, int64_t n_targets, int64_t n_mids, int32_t tile_w,
                       const uint32_t* tile_off, const uint32_t* tile_ent,
                       const uint32_t* tile_maxc, const int64_t* tile_gmin,
                       const dps_cct_ext* ext, int64_t row_begin,
                       int64_t row_end, const int32_t* row_order, int64_t n_order,
                       const int32_t* piece_t0, const int32_t* piece_t1, int64_t n_pieces,
                       int32_t* piece_idx, int64_t* piece_cnt, double* piece_score, int32_t k,
                       int32_t* out_idx, int64_t* out_cnt, double* out_score, void* ws,
                       size_t ws_bytes, void* stream) {
  DPS_REQUIRE(0 <= row_begin && row_begin <= row_end && row_end <= n_targets, DPS_ERR_INVALID,
              "row range [%lld, %lld) outside [0, %lld)", static_cast<long long>(row_begin),
              static_cast<long long>(row_end), static_cast<long long>(n_targets));
  DPS_REQUIRE(n_pieces >= 0 && n_order >= n_pieces, DPS_ERR_INVALID, "bad n_order / n_pieces");
  DPS_REQUIRE(n_order - n_pieces <= row_end - row_begin, DPS_ERR_INVALID,
              "more whole rows than the range holds");
  DPS_REQUIRE(n_order == 0 || row_order, DPS_ERR_INVALID, "row_order is required");
  DPS_REQUIRE(n_pieces == 0 || (piece_t0 && piece_t1 && piece_idx && piece_cnt && piece_score),
              DPS_ERR_INVALID, "piece ranges and outputs are required");
  return cct_topk_impl(c_ptr, c_col, c_val, g, g_t, t_perm, t_rank, n_targets, n_mids, tile_w,
                       tile_off, tile_ent, tile_maxc, tile_gmin, ext, row_begin, n_order,
                       row_order, false, k, out_idx, out_cnt, out_score, ws, ws_bytes, stream, n_pieces,
                       piece_t0, piece_t1, piece_idx, piece_cnt, piece_score);
}

size_t dps_cct_sym_workspace_size(int64_t n_targets, int32_t k, int64_t rec_cap) {
  const size_t n = static_cast<size_t>(n_targets > 0 ? n_targets : 1);
  const size_t nk = n * static_cast<size_t>(k > 0 ? k : 1);
  const size_t cap = static_cast<size_t>(rec_cap > 0 ? rec_cap : 1);
  size_t b = 0;
  b += align_up(nk * 4) + align_up(nk * 8) + align_up(nk * 8);   // rest lists
  b += align_up(n) + align_up(n * 4) + align_up((n / 2048 + 2) * 4);   // strong, tau_emit, tau_blk
  b += 2 * align_up((n + 1) * 4) + align_up((n / 2048 + 2) * 4);   // tau_tile, tile_done, blk_done
  b += align_up(n * 4);                                          // rest-pass order
  b += 5 * align_up(cap * 4);                                    // records + placed records
  b += align_up(8) + 2 * align_up((n + 1) * 4) + align_up((n + 1) * 8);
  b += align_up(scan_workspace_size(n_targets + 1)) + align_up(dps_cct_topk_workspace_size());
  return b + 1024;
}

int dps_cct_sym(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                const int64_t* g, const int64_t* g_t, const int32_t* t_perm,
                const int32_t* t_rank, int64_t n_targets, int64_t n_mids, int32_t tile_w,
                const uint32_t* tile_off, const uint32_t* tile_ent, const uint32_t* tile_maxc,
                const int64_t* tile_gmin, const dps_cct_ext* ext, const int32_t* row_order,
                int32_t band, int64_t rec_cap, int32_t k, int32_t* out_idx, int64_t* out_cnt,
                double* out_score, unsigned long long* rec_stat, void* sym_ws, size_t sym_ws_bytes,
                void* ws, size_t ws_bytes, void* stream) {
  DPS_REQUIRE(band >= 0 && band <= 64, DPS_ERR_INVALID, "band must be in [0, 64]");
  DPS_REQUIRE(rec_cap >= 1 && rec_cap < (int64_t(1) << 40), DPS_ERR_INVALID, "bad rec_cap");
  DPS_REQUIRE(k >= 1 && k <= 256, DPS_ERR_UNSUPPORTED, "k must be in [1, 256], got %d", k);
  DPS_REQUIRE(n_targets >= 0 && n_targets < INT32_MAX, DPS_ERR_OVERFLOW, "bad n_targets");
  DPS_REQUIRE(rec_stat && out_idx && out_cnt && out_score, DPS_ERR_INVALID, "null output");
  DPS_REQUIRE(ext == nullptr || ext->s == nullptr, DPS_ERR_UNSUPPORTED,
              "symmetric mode runs without venue skipping");
  DPS_REQUIRE(reinterpret_cast<uintptr_t>(sym_ws) % 256 == 0, DPS_ERR_WORKSPACE,
              "workspace not 256-byte aligned");
  DPS_REQUIRE(sym_ws_bytes >= dps_cct_sym_workspace_size(n_targets, k, rec_cap),
              DPS_ERR_WORKSPACE, "cct_sym workspace too small");
  auto st = static_cast<hipStream_t>(stream);
  const int64_t n = n_targets;
  if (n == 0) return DPS_OK;
  const int shift = log2_exact(tile_w);
  DPS_REQUIRE(shift == 13 || shift == 14, DPS_ERR_UNSUPPORTED,
              "symmetric mode needs tile_w 8192 or 16384, got %d", tile_w);
  const int64_t T = (n + tile_w - 1) / tile_w;
  const int64_t nk = n * k;
  Carve c(sym_ws, sym_ws_bytes);
  int32_t* r_idx = c.take<int32_t>(nk);
  int64_t* r_cnt = c.take<int64_t>(nk);
  double* r_score = c.take<double>(nk);
  uint8_t* strong = c.take<uint8_t>(n);
  float* tau_emit = c.take<float>(n);
  uint32_t* tau_blk = c.take<uint32_t>(n / 2048 + 2);
  uint32_t* tau_tile = c.take<uint32_t>(T + 1);
  uint32_t* blk_done = c.take<uint32_t>(n / 2048 + 2);
  uint32_t* tile_done = c.take<uint32_t>(T + 1);
  int32_t* dq = c.take<int32_t>(n);
  int32_t* rec_y = c.take<int32_t>(rec_cap);
  int32_t* rec_x = c.take<int32_t>(rec_cap);
  int32_t* rec_m = c.take<int32_t>(rec_cap);
  int32_t* sx = c.take<int32_t>(rec_cap);
  int32_t* sm = c.take<int32_t>(rec_cap);
  unsigned long long* rec_n = c.take<unsigned long long>(1);
  uint32_t* cnt = c.take<uint32_t>(n + 1);
  uint32_t* cur = c.take<uint32_t>(n + 1);
  int64_t* off = c.take<int64_t>(n + 1);
  const size_t scan_ws = scan_workspace_size(n + 1);
  void* sws = c.take<char>(scan_ws);
  // (the hot kernel's counter words, dps_cct_topk_workspace_size bytes)
  unsigned long long* band_ctr =
      c.take<unsigned long long>(dps_cct_topk_workspace_size() / sizeof(unsigned long long));
  DPS_REQUIRE(c.ok, DPS_ERR_WORKSPACE, "cct_sym workspace carve failed");
  {
    FillSet fs;
    fs.add(tau_blk, n / 2048 + 2, 0x7F800000u);   // +inf
    fs.add(tau_tile, T + 1, 0x7F800000u);
    fs.add(blk_done, n / 2048 + 2, 0u);
    fs.add(tile_done, T + 1, 0u);
    fs.add(reinterpret_cast<uint32_t*>(rec_n), 2, 0u);
    fs.add(cnt, n + 1, 0u);
    fs.add(cur, n + 1, 0u);
    DPS_HIP_RET(fill_set(fs, st));
  }
  SymSetup sy{};
  sy.band = band;
  // 1. band pass: every row over its own tile +- band, into out_*
  sy.sym = 1;
  int rc = cct_topk_impl(c_ptr, c_col, c_val, g, g_t, t_perm, t_rank, n, n_mids, tile_w, tile_off,
                         tile_ent, tile_maxc, tile_gmin, ext, 0, n, row_order, false, k, out_idx,
                         out_cnt, out_score, band_ctr, dps_cct_topk_workspace_size(), stream, 0,
                         nullptr, nullptr, nullptr,
                         nullptr, nullptr, &sy);
  if (rc != DPS_OK) return rc;
  // 2. plan: strong rows and the emission thresholds
  k_sym_plan<<<grid_for(n, 256), 256, 0, st>>>(n, k, shift, t_rank, out_score, strong, tau_emit,
                                                 tau_blk, tau_tile);
  DPS_LAUNCHED();
  // rest pass in descending label order: a row's far targets (higher labels)
  // have mostly finished and published their own k-th scores by then
  k_desc_order<<<grid_for(n, 256), 256, 0, st>>>(t_perm, n, dq);
  DPS_LAUNCHED();
  // 3. rest pass: records for the pairs only this row sees
  sy.sym = 2;
  sy.row_strong = strong;
  sy.seed_idx = out_idx;
  sy.seed_score = out_score;
  sy.tau_emit = tau_emit;
  sy.tau_blk = reinterpret_cast<float*>(tau_blk);
  sy.tau_tile = reinterpret_cast<float*>(tau_tile);
  sy.blk_done = blk_done;
  sy.tile_done = tile_done;
  sy.rec_y = rec_y; sy.rec_x = rec_x; sy.rec_m = rec_m;
  sy.rec_n = rec_n; sy.rec_cap = rec_cap;
  rc = cct_topk_impl(c_ptr, c_col, c_val, g, g_t, t_perm, t_rank, n, n_mids, tile_w, tile_off,
                     tile_ent, tile_maxc, tile_gmin, ext, 0, n, dq, false, k, r_idx, r_cnt, r_score,
                     ws, ws_bytes, stream, 0, nullptr, nullptr, nullptr, nullptr, nullptr, &sy);
  if (rc != DPS_OK) return rc;
  k_add_counts<<<1, 64, 0, st>>>(band_ctr, static_cast<unsigned long long*>(ws));
  DPS_LAUNCHED();
  // 4. records grouped by target row, then the final lists
  k_rec_count<<<grid_for(rec_cap, 256), 256, 0, st>>>(rec_y, rec_n, rec_cap, cnt);
  DPS_LAUNCHED();
  DPS_HIP_RET(scan_exclusive<uint32_t>(cnt, off, n + 1, sws, scan_ws, st));
  k_rec_place<<<grid_for(rec_cap, 256), 256, 0, st>>>(rec_y, rec_x, rec_m, rec_n, rec_cap, off, cur,
                                                       sx, sm);
  DPS_LAUNCHED();
  const unsigned grid = static_cast<unsigned>((n + 3) / 4 < 4096 ? (n + 3) / 4 : 4096);
  if (k <= 64)
    k_sym_merge<1><<<grid, 256, 0, st>>>(n, k, strong, g, r_idx, r_cnt, r_score, off, sx, sm,
                                          out_idx, out_cnt, out_score);
  else if (k <= 128)
    k_sym_merge<2><<<grid, 256, 0, st>>>(n, k, strong, g, r_idx, r_cnt, r_score, off, sx, sm,
                                          out_idx, out_cnt, out_score);
  else
    k_sym_merge<4><<<grid, 256, 0, st>>>(n, k, strong, g, r_idx, r_cnt, r_score, off, sx, sm,
                                          out_idx, out_cnt, out_score);
  DPS_LAUNCHED();
  // records emitted (may exceed rec_cap: then the lists are incomplete and the
  // caller must rerun with a larger capacity)
  DPS_HIP_RET(hipMemcpyAsync(rec_stat, rec_n, sizeof(unsigned long long), hipMemcpyDeviceToDevice, st));
  return DPS_OK;
}

int dps_topk_merge(const int32_t* piece_idx, const int64_t* piece_cnt, const double* piece_score,
                   const int32_t* rows, int64_t n_groups, int32_t pieces_per_row, int32_t k,
                   int64_t n_targets, int64_t row_begin, int32_t* out_idx, int64_t* out_cnt,
                   double* out_score, void* stream) {
  DPS_REQUIRE(n_groups >= 0 && pieces_per_row >= 1 && pieces_per_row <= kWave, DPS_ERR_INVALID,
              "pieces_per_row must be in [1, 64]");
  DPS_REQUIRE(k >= 1 && k <= kMergeMaxK, DPS_ERR_UNSUPPORTED, "k must be in [1, 256]");
  if (n_groups == 0) return DPS_OK;
  DPS_REQUIRE(piece_idx && piece_cnt && piece_score && rows && out_idx && out_cnt && out_score,
              DPS_ERR_INVALID, "null array");
  auto st = static_cast<hipStream_t>(stream);
  const unsigned grid = static_cast<unsigned>((n_groups + 3) / 4 < 2048 ? (n_groups + 3) / 4 : 2048);
  k_topk_merge<<<grid, 256, 0, st>>>(piece_idx, piece_cnt, piece_score, rows, n_groups,
                                     pieces_per_row, k, n_targets, row_begin, out_idx, out_cnt,
                                     out_score);
  DPS_LAUNCHED();
  return DPS_OK;
}

}  // extern "C"
