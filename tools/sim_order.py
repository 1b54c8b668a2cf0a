"""Simulation (CPU, numpy): target tiles the hot kernel scans per row under
different tile orders.

The kernel skips tile t of row x when UB[x,t] = sum_v C[x,v] * maxc[v,t] is
below mneed(tau, gx + gmin_t), tau = the k-th best score over the tiles
scanned so far.  The order in which tiles are visited decides how fast tau
rises.  Policies compared (each row simulated exactly from its M row):
  asc      ascending g (the round-2 kernel)
  bestub   descending score bound 2 UB / (gx + gmin_t)
  near     tiles ordered by |centre g - gx| (targets like x first)
  seedK    K tiles of largest UB*... first, then ascending
  oracle   the final tau known before the sweep (lower bound)
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
nrows = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
W = int(os.environ.get("SIM_W", "8192"))
t0 = time.time()
g = synth_config(cfg)
t = g.typed()
co = po.COracle.from_typed(t)
cp, cc, cv, s, gg = co.export()
NA, NV = t.n_authors, t.n_mids
cp = cp[: NA + 1]
cc = cc[: cp[-1]]
cv = cv[: cp[-1]]
print(f"{cfg}: NA={NA} nnz={len(cc)} build {time.time()-t0:.1f}s", flush=True)
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
g_lab = gg[order]
gmin = g_lab[np.arange(T) * W]
gctr = g_lab[np.minimum(np.arange(T) * W + W // 2, NA - 1)]

rng = np.random.default_rng(7)
rows = np.sort(rng.choice(NA, size=nrows, replace=False))


def mneed(tau, den):
    if tau <= 0:
        return 0
    return int(np.ceil(tau * den * 0.5 * (1 - 2.0 ** -40)))


LAMS = (0.0, 0.25, 0.5, 0.75, 1.0)


def witness_skip(tau, tt, a, sv, mx, gx):
    """True if sum_v maxc[v,t] * max(0, 2 a_v - tau (1-lam) s_v) < tau (gx + lam gmin_t)
    for some lam (then no target of tile t scores >= tau)."""
    tt_ = tau * (1 - 2.0 ** -40)
    for lam in LAMS:
        coef = np.maximum(0.0, 2.0 * a - tt_ * (1 - lam) * sv)
        if (mx[:, tt] * coef).sum() < tt_ * (gx + lam * gmin[tt]):
            return True
    return False


def simulate(ub, tile_best, order_t, gx, tau_fixed=None, wit=None):
    """tile_best[t] = sorted desc scores of the tile's targets (k best)."""
    best = np.full(k, -1.0)
    scanned = 0
    for tt in order_t:
        tau = tau_fixed if tau_fixed is not None else (best[k - 1] if best[k - 1] >= 0 else -1.0)
        if ub[tt] == 0:
            continue
        if tau > 0 and ub[tt] < mneed(tau, gx + gmin[tt]):
            continue
        if wit is not None and tau > 0 and witness_skip(tau, tt, *wit, gx):
            continue
        scanned += 1
        allb = np.concatenate([best, tile_best[tt]])
        best = -np.sort(-allb)[:k]
    return scanned


pol = {"asc": 0, "bestub": 0, "oracle": 0, "w_asc": 0, "w_desc": 0, "w_near": 0, "w_oracle": 0,
       "nonempty": 0}
tb0 = time.time()
for i0 in range(0, nrows, 100):
    rr = rows[i0:i0 + 100]
    Mb = (C[rr] @ CT).tocsr()
    for j, x in enumerate(rr):
        m = Mb.getrow(j)
        y, mv = m.indices, m.data
        keep = y != x
        y, mv = y[keep], mv[keep]
        gx = int(gg[x])
        sc = 2.0 * mv / (gx + gg[y]).astype(np.float64)
        lab = rank[y]
        tl = lab // W
        # per tile: top-k scores
        o = np.lexsort((-sc, tl))
        tl_s, sc_s = tl[o], sc[o]
        starts = np.searchsorted(tl_s, np.arange(T))
        ends = np.searchsorted(tl_s, np.arange(T), side="right")
        tile_best = []
        for tt in range(T):
            b = sc_s[starts[tt]:min(ends[tt], starts[tt] + k)]
            tile_best.append(np.pad(b, (0, k - len(b)), constant_values=-1.0))
        b0, b1 = cp[x], cp[x + 1]
        ub = (cv[b0:b1, None].astype(np.int64) * maxc[cc[b0:b1]]).sum(0)
        allsc = np.sort(sc)[::-1]
        tau_final = allsc[k - 1] if len(allsc) >= k else -1.0
        pol["nonempty"] += int((ub > 0).sum())
        asc = np.arange(T)
        pol["asc"] += simulate(ub, tile_best, asc, gx)
        bound = 2.0 * ub / (gx + gmin)
        pol["bestub"] += simulate(ub, tile_best, np.argsort(-bound, kind="stable"), gx)
        pol["oracle"] += simulate(ub, tile_best, asc, gx, tau_fixed=tau_final)
        wit = (cv[b0:b1].astype(np.float64), s[cc[b0:b1]].astype(np.float64),
               maxc[cc[b0:b1]].astype(np.float64))
        pol["w_asc"] += simulate(ub, tile_best, asc, gx, wit=wit)
        pol["w_desc"] += simulate(ub, tile_best, asc[::-1], gx, wit=wit)
        pol["w_near"] += simulate(ub, tile_best, np.argsort(np.abs(gctr - gx), kind="stable"), gx, wit=wit)
        pol["w_oracle"] += simulate(ub, tile_best, asc, gx, tau_fixed=tau_final, wit=wit)
    print(f"{i0+len(rr)} rows {time.time()-tb0:.0f}s " +
          " ".join(f"{kk}={v/(i0+len(rr)):.1f}" for kk, v in pol.items()), flush=True)
