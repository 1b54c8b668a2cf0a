"""Simulation (CPU, numpy): tiles the hot kernel scans per row under tighter
per-tile bounds.

Targets are relabelled by ascending g and cut into tiles of W labels (the
kernel's layout).  Tile t of row x is skipped when its bound B[x,t] on
max_{y in t} M[x,y] is below mneed(tau, gx + gmin_t).  Bounds compared:
  ub    sum_v C[x,v] * maxc[v,t]                       (the round-2 kernel)
  cs    floor(sqrt(M[x,x] * max_{y in t} M[y,y]))      (Cauchy-Schwarz)
  l1    max_v C[x,v] * max_{y in t} |C[y,:]|_1          (Hoelder 1/inf)
  min   min(ub, cs, l1)
each with the running tau (ascending tile order) and with the final tau.
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
nrows = int(sys.argv[3]) if len(sys.argv) > 3 else 500
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
dg = np.asarray(C.multiply(C).sum(1)).ravel().astype(np.int64)
l1 = np.asarray(C.sum(1)).ravel().astype(np.int64)
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
lab_tile = rank // W
maxdg = np.zeros(T, np.int64)
np.maximum.at(maxdg, lab_tile, dg)
maxl1 = np.zeros(T, np.int64)
np.maximum.at(maxl1, lab_tile, l1)
g_lab = gg[order]
gmin = g_lab[np.arange(T) * W]

rng = np.random.default_rng(7)
rows = np.sort(rng.choice(NA, size=nrows, replace=False))


def scanned(bound, tile_best, gx, tau_fixed=None, chunks=None):
    best = np.full(k, -1.0)
    n = 0
    nch = 0
    for tt in range(T):
        tau = tau_fixed if tau_fixed is not None else best[k - 1]
        if bound[tt] == 0:
            continue
        if tau > 0 and bound[tt] < np.ceil(tau * (gx + gmin[tt]) * 0.5 * (1 - 2.0 ** -40)):
            continue
        n += 1
        if chunks is not None:
            nch += chunks[tt]
        best = -np.sort(-np.concatenate([best, tile_best[tt]]))[:k]
    if chunks is not None:
        res["chunks"] += nch
    return n


names = ("ub", "cs", "l1", "min")
res = {f"{nm}{suf}": 0 for nm in names for suf in ("", "_oracle")}
res["perfect"] = 0
res["chunks"] = 0
tb0 = time.time()
for i0 in range(0, nrows, 50):
    rr = rows[i0:i0 + 50]
    Mb = (C[rr] @ CT).tocsr()
    for j, x in enumerate(rr):
        m = Mb.getrow(j)
        y, mv = m.indices, m.data
        keep = y != x
        y, mv = y[keep], mv[keep]
        gx = int(gg[x])
        sc = 2.0 * mv / (gx + gg[y]).astype(np.float64)
        tl = rank[y] // W
        o = np.lexsort((-sc, tl))
        tl_s, sc_s = tl[o], sc[o]
        st = np.searchsorted(tl_s, np.arange(T))
        en = np.searchsorted(tl_s, np.arange(T), side="right")
        tile_best = [np.pad(sc_s[st[q]:min(en[q], st[q] + k)], (0, k - min(en[q] - st[q], k)),
                            constant_values=-1.0) for q in range(T)]
        tmax = np.zeros(T, np.int64)
        np.maximum.at(tmax, tl, mv)
        b0, b1 = cp[x], cp[x + 1]
        ub = (cv[b0:b1, None].astype(np.int64) * maxc[cc[b0:b1]]).sum(0)
        cs = np.floor(np.sqrt(dg[x].astype(np.float64) * maxdg)).astype(np.int64)
        hl = int(cv[b0:b1].max()) * maxl1
        bd = {"ub": ub, "cs": cs, "l1": hl, "min": np.minimum(np.minimum(ub, cs), hl)}
        allsc = np.sort(sc)[::-1]
        tau_final = allsc[k - 1] if len(allsc) >= k else -1.0
        chunks = ((bcnt[cc[b0:b1]] + 7) // 8).sum(0)
        for nm in names:
            res[nm] += scanned(bd[nm], tile_best, gx, chunks=chunks if nm == "ub" else None)
            res[nm + "_oracle"] += scanned(bd[nm], tile_best, gx, tau_fixed=tau_final)
        res["perfect"] += scanned(tmax, tile_best, gx, tau_fixed=tau_final)
    nn = i0 + len(rr)
    print(f"W={W} slots/row ub {res['ub']*W/nn:.0f} chunks/row {res['chunks']/nn:.0f}")
    print(f"{nn} rows {time.time()-tb0:.0f}s " + " ".join(f"{kk}={v/nn:.1f}" for kk, v in res.items()),
          flush=True)
