"""Simulation (CPU, numpy): the top-D tile bound.

ub[x,t]  = sum_v a_v maxc[v,t]  (the kernel's bound, a_v = C[x,v]) assumes one
target of tile t holds the maximum count in EVERY venue of x.  A target y has
at most deg(y) venues, so with D_t = max_{y in t} deg(y)
   M[x,y] <= sum of the D_t largest a_v maxc[v,t]   =: ubD[x,t].
Reports tiles per row whose bound reaches mneed(tau_final, gx + gmin_t), for
ub, ubD and perfect (tiles holding a target that scores >= tau_final), over a
row sample stratified by row work.
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
W = int(os.environ.get("SIM_W", "16384"))
t0 = time.time()
t = synth_config(cfg).typed()
co = po.COracle.from_typed(t)
cp, cc, cv, s, gg = co.export()
NA, NV = t.n_authors, t.n_mids
cp = cp[: NA + 1]
cc = cc[: cp[-1]]
cv = cv[: cp[-1]].astype(np.int64)
gg = gg[:NA].astype(np.int64)
print(f"{cfg}: NA={NA} nnz={len(cc)} build {time.time()-t0:.1f}s", flush=True)
C = sp.csr_matrix((cv, cc, cp), shape=(NA, NV))
CT = C.T.tocsr()
order = np.argsort(gg, kind="stable")
rank = np.empty(NA, np.int64)
rank[order] = np.arange(NA)
T = (NA + W - 1) // W
g_lab = gg[order]
gmin = g_lab[np.arange(T) * W]
row_of = np.repeat(np.arange(NA), np.diff(cp))
tile_of_row = rank // W
maxc = np.zeros((NV, T), np.int64)
np.maximum.at(maxc, (cc, tile_of_row[row_of]), cv)
deg = np.diff(cp)
D = np.zeros(T, np.int64)
np.maximum.at(D, tile_of_row, deg)
print("max degree per tile (first 8, last 8):", D[:8].tolist(), D[-8:].tolist(), flush=True)
n_v = np.bincount(cc, minlength=NV)
terms = np.asarray(C @ sp.csr_matrix(n_v[:, None].astype(np.int64))).ravel() if False else \
    np.add.reduceat(n_v[cc], cp[:-1]) * (deg > 0)
rng = np.random.default_rng(7)
qs = np.quantile(terms, [0.0, 0.33, 0.66, 1.0])
res = {}
for band in range(3):
    pool = np.flatnonzero((terms >= qs[band]) & (terms <= qs[band + 1]) & (deg > 0))
    rows = rng.choice(pool, min(nrows, len(pool)), replace=False)
    acc = np.zeros(4)
    for x in rows:
        a0, a1 = cp[x], cp[x + 1]
        v, a = cc[a0:a1], cv[a0:a1]
        mrow = np.asarray((CT[v].T @ a)).ravel() if False else np.asarray(C @ sp.csr_matrix(
            (a, v, [0, len(v)]), shape=(1, NV)).T.todense()).ravel()
        mrow[x] = 0
        den = (gg[x] + gg).astype(np.float64)
        sc = 2.0 * mrow / den
        tau = np.sort(sc)[-k]
        if tau <= 0:
            continue
        mneed = np.ceil(tau * (gg[x] + gmin) / 2.0 - 1e-9)
        prod = a[:, None] * maxc[v]                      # [d, T]
        ub = prod.sum(0)
        ps = -np.sort(-prod, axis=0)                     # descending per tile
        cs = np.cumsum(ps, 0)
        dd = np.minimum(D, len(v)) - 1
        ubd = cs[dd, np.arange(T)]
        lab_tile = tile_of_row[np.flatnonzero(sc >= tau)]
        perfect = len(np.unique(lab_tile))
        acc += [(ub >= mneed).sum(), (ubd >= mneed).sum(), perfect, 1]
    res[band] = acc
    n = acc[3]
    print(f"row-work band {band} (terms {qs[band]:.0f}..{qs[band+1]:.0f}), {int(n)} rows: tiles/row "
          f"ub {acc[0]/n:.1f}  ubD {acc[1]/n:.1f}  perfect {acc[2]/n:.1f}  of {T}", flush=True)
print(f"done {time.time()-t0:.0f}s")
