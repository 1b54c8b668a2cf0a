"""Simulation (CPU, numpy): the hot kernel with venue skipping.

Every target y has g[y] = sum_u C[y,u] s_u >= sum_{v in x} C[y,v] s_v.  Split the
venues of row x at the current k-th score tau into
  Q = {v : 2 a_v > tau s_v}   (qualifying)   and   H = the rest,
a_v = C[x,v], b_v = C[y,v], rho_H = max_{v in H} a_v / s_v (<= tau / 2).  Then
  M_H(y) = sum_{v in H} a_v b_v <= rho_H * sum_{v in H} b_v s_v <= rho_H * g[y],
so score(y) >= tau needs  M_Q(y) >= tau gx / 2 + (tau / 2 - rho_H) g[y].
The kernel then scatters only the Q venues' buckets of a tile, flags targets by
that test (per 1024-target segment with the segment's smallest g), and
computes the exact M of each flagged target from the two C rows ("verify").
Tiles are skipped when sum_{v in Q} a_v maxc[v,t] is below the test's right side
at gmin_t.  Q is re-derived per tile from the running tau (tiles ascending).

Reported per row: tiles scanned, 16-byte chunks scattered, candidates
verified, against the round-2 kernel (every venue, UB tile skip).
"""
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "distributed-pathsim_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
from dpathsim.synth import synth_config  # noqa: E402
import pathsim_oracle as po  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "config3"
k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
nrows = int(sys.argv[3]) if len(sys.argv) > 3 else 200
W = int(os.environ.get("SIM_W", "8192"))
SEG = 1024
KH = int(os.environ.get("SIM_KH", "0"))
TIGHT = int(os.environ.get("SIM_TIGHT", "0"))   # also bound M_H by sum_{h in H} a_h maxc[h,t]     # H restricted to the KH venues of largest n_v (0: any)
t0 = time.time()
g = synth_config(cfg)
t = g.typed()
co = po.COracle.from_typed(t)
cp, cc, cv, s, gg = co.export()
NA, NV = t.n_authors, t.n_mids
cp = cp[: NA + 1]
cc = cc[: cp[-1]]
cv = cv[: cp[-1]]
s = s.astype(np.float64)
gg = gg[:NA].astype(np.int64)
C = sp.csr_matrix((cv.astype(np.int64), cc, cp), shape=(NA, NV))
CT = C.T.tocsr()
order = np.argsort(gg, kind="stable")
rank = np.empty(NA, np.int64)
rank[order] = np.arange(NA)
T = (NA + W - 1) // W
row_of = np.repeat(np.arange(NA), np.diff(cp))
tile_of_entry = rank[row_of] // W
maxc = np.zeros((NV, T), np.int64)
np.maximum.at(maxc, (cc, tile_of_entry), cv)
bcnt = np.zeros((NV, T), np.int64)
np.add.at(bcnt, (cc, tile_of_entry), 1)
g_lab = gg[order].astype(np.float64)
gmin = g_lab[np.arange(T) * W]
nseg = (NA + SEG - 1) // SEG
gseg = g_lab[np.arange(nseg) * SEG]
nv_cnt = np.bincount(cc, minlength=NV)
heavy = np.zeros(NV, bool)
if KH > 0:
    heavy[np.argsort(-nv_cnt, kind="stable")[:KH]] = True
else:
    heavy[:] = True
print(f"{cfg}: NA={NA} nnz={len(cc)} tables {time.time()-t0:.1f}s W={W} KH={KH}", flush=True)

rng = np.random.default_rng(7)
rows = np.sort(rng.choice(NA, size=nrows, replace=False))
EPS = 1 - 2.0 ** -40


def better_insert(best_s, best_y, sc, yy):
    s2 = np.concatenate([best_s, sc])
    y2 = np.concatenate([best_y, yy])
    o = np.lexsort((y2, -s2))[:k]
    return s2[o], y2[o]


res = {"old_tiles": 0, "old_chunks": 0, "tiles": 0, "chunks": 0, "verify": 0, "qfrac": 0.0,
       "hv_tiles": 0, "mism": 0, "nib": 0, "u8": 0, "old_cand": 0, "cand": 0}
tb0 = time.time()
for i0 in range(0, nrows, 25):
    rr = rows[i0:i0 + 25]
    for x in rr:
        b0, b1 = cp[x], cp[x + 1]
        vx = cc[b0:b1]
        a = cv[b0:b1].astype(np.float64)
        sv = s[vx]
        gx = float(gg[x])
        # per (venue j of x, target) contributions
        ys, js, bs = [], [], []
        for j, v in enumerate(vx):
            lo, hi = CT.indptr[v], CT.indptr[v + 1]
            ys.append(CT.indices[lo:hi])
            bs.append(CT.data[lo:hi])
            js.append(np.full(hi - lo, j))
        ys = np.concatenate(ys)
        js = np.concatenate(js)
        bs = np.concatenate(bs).astype(np.float64)
        keep = ys != x
        ys, js, bs = ys[keep], js[keep], bs[keep]
        lab = rank[ys]
        tl = lab // W
        Mfull = np.bincount(ys, weights=a[js] * bs, minlength=0)
        # reference answer (exact top-k)
        yu = np.unique(ys)
        sc_all = 2.0 * Mfull[yu] / (gx + gg[yu])
        ref_s, ref_y = better_insert(np.full(0, -1.0), np.zeros(0, np.int64), sc_all, yu)
        # group entries by tile
        o = np.argsort(tl, kind="stable")
        ys, js, bs, lab, tl = ys[o], js[o], bs[o], lab[o], tl[o]
        st = np.searchsorted(tl, np.arange(T + 1))
        # --- round-2 kernel: all venues, UB skip
        best_s = np.full(k, -1.0)
        best_y = np.full(k, -1, np.int64)
        ub = (a[:, None] * maxc[vx]).sum(0)
        ch = ((bcnt[vx] + 7) // 8)
        for tt in range(T):
            tau = best_s[k - 1]
            if ub[tt] == 0:
                continue
            if tau > 0 and ub[tt] < np.ceil(tau * (gx + gmin[tt]) * 0.5 * EPS):
                continue
            res["old_tiles"] += 1
            res["old_chunks"] += ch[:, tt].sum()
            e = slice(st[tt], st[tt + 1])
            yy = np.unique(ys[e])
            if tau > 0:
                gs = gseg[rank[yy] // SEG]
                ok = Mfull[yy] >= np.ceil(tau * (gx + gs) * 0.5 * EPS - 1e-9)
                res["old_cand"] += int(ok.sum())
                yy = yy[ok]
            else:
                res["old_cand"] += len(yy)
            scy = 2.0 * Mfull[yy] / (gx + gg[yy])
            best_s, best_y = better_insert(best_s, best_y, scy, yy)
        # --- venue skipping
        best_s = np.full(k, -1.0)
        best_y = np.full(k, -1, np.int64)
        for tt in range(T):
            tau = best_s[k - 1]
            if tau > 0:
                q = (2.0 * a > tau * sv * EPS) | ~heavy[vx]
            else:
                q = np.ones(len(a), bool)
            rho = float((a[~q] / sv[~q]).max()) if (~q).any() else 0.0
            coef = max(tau / 2 - rho, 0.0) if tau > 0 else 0.0
            ubq = (a[q, None] * maxc[vx[q], tt:tt + 1]).sum() if q.any() else 0
            if ubq == 0:
                continue
            if tau > 0 and ubq < tau * gx / 2 * EPS + coef * gmin[tt] * EPS:
                continue
            res["tiles"] += 1
            res["nib"] += ubq <= 15
            res["u8"] += ubq <= 255
            res["qfrac"] += q.mean()
            res["chunks"] += ch[q, tt].sum()
            e = slice(st[tt], st[tt + 1])
            qe = q[js[e]]
            yq = ys[e][qe]
            if len(yq) == 0:
                continue
            MQ = np.bincount(yq, weights=a[js[e][qe]] * bs[e][qe])
            yy = np.unique(yq)
            mq = MQ[yy]
            if tau <= 0:
                res["cand"] += len(yy)
            if tau > 0:
                gs = gseg[rank[yy] // SEG]
                thr = tau * gx / 2 * EPS + coef * gs * EPS
                if TIGHT and (~q).any():
                    # M_H(y) <= sum_{h in H} a_h maxc[h, t] as well
                    ubh = float((a[~q] * maxc[vx[~q], tt]).sum())
                    thr = np.maximum(thr, np.ceil(tau * (gx + gs) * 0.5 * EPS) - ubh)
                cand = mq >= np.ceil(thr - 1e-9)
                res["cand"] += int(cand.sum())
                if (~q).any():
                    res["hv_tiles"] += 1
                    res["verify"] += int(cand.sum())
                yy = yy[cand]
            scy = 2.0 * Mfull[yy] / (gx + gg[yy])
            best_s, best_y = better_insert(best_s, best_y, scy, yy)
        if not (np.array_equal(best_y, ref_y[:k]) and np.array_equal(best_s, ref_s[:k])):
            res["mism"] += 1
    nn = i0 + len(rr)
    print(f"{nn} rows {time.time()-tb0:.0f}s  " +
          " ".join(f"{kk}={v/nn:.2f}" for kk, v in res.items()), flush=True)
