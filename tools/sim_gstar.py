"""Simulation (CPU, numpy): the g-threshold implied by rho_x.

M[x,y] = sum_v (C[x,v]/s_v) C[y,v] s_v <= rho_x g[y] with rho_x = max_v C[x,v]/s_v,
so score(y) = 2M/(gx+gy) >= tau needs gy (2 rho_x - tau) >= tau gx, i.e.
gy >= g* = tau gx / (2 rho_x - tau).  Targets are relabelled by ascending g,
so every tile whose largest g is below g* can be skipped.  Reports, per row,
tiles (W = SIM_W) with gmax < g* under the final tau, and the terms of those
tiles, against the tiles the ub bound already skips.
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
nrows = int(sys.argv[3]) if len(sys.argv) > 3 else 300
W = int(os.environ.get("SIM_W", "16384"))
t0 = time.time()
t = synth_config(cfg).typed()
co = po.COracle.from_typed(t)
cp, cc, cv, s, gg = co.export()
NA, NV = t.n_authors, t.n_mids
cp = cp[: NA + 1]
cc = cc[: cp[-1]]
cv = cv[: cp[-1]]
gg = gg[:NA].astype(np.int64)
s = s[:NV].astype(np.int64)
print(f"{cfg}: NA={NA} nnz={len(cc)} build {time.time()-t0:.1f}s", flush=True)
C = sp.csr_matrix((cv.astype(np.int64), cc, cp), shape=(NA, NV))
order = np.argsort(gg, kind="stable")
rank = np.empty(NA, np.int64)
rank[order] = np.arange(NA)
T = (NA + W - 1) // W
g_lab = gg[order]
gmax = g_lab[np.minimum((np.arange(T) + 1) * W, NA) - 1]
gmin = g_lab[np.arange(T) * W]
row_of = np.repeat(np.arange(NA), np.diff(cp))
maxc = np.zeros((NV, T), np.int64)
np.maximum.at(maxc, (cc, rank[row_of] // W), cv)
rng = np.random.default_rng(1)
rows = rng.choice(NA, nrows, replace=False)
tot_skip = tot_ub = tot_both = 0
frac_lab = []
for i, x in enumerate(rows):
    a0, a1 = cp[x], cp[x + 1]
    if a1 == a0:
        continue
    v, c = cc[a0:a1], cv[a0:a1].astype(np.int64)
    m = np.asarray(C @ sp.csr_matrix((c, v, [0, len(v)]), shape=(1, NV)).T.todense()).ravel()
    m[x] = 0
    den = (gg[x] + gg).astype(np.float64)
    sc = np.where(den > 0, 2.0 * m / np.where(den > 0, den, 1), 0.0)
    sc[x] = -1
    tau = np.sort(sc)[-k]
    rho = float(np.max(c / s[v]))
    if tau <= 0 or 2 * rho <= tau:
        gstar = np.inf if tau > 0 else 0
    else:
        gstar = tau * gg[x] / (2 * rho - tau)
    skip_g = gmax < gstar
    ub = (c[:, None] * maxc[v]).sum(0)
    need = tau * (gg[x] + gmin) / 2
    skip_ub = ub < need
    tot_skip += skip_g.sum(); tot_ub += skip_ub.sum(); tot_both += (skip_g | skip_ub).sum()
    frac_lab.append(np.searchsorted(g_lab, gstar) / NA if np.isfinite(gstar) else 1.0)
    if (i + 1) % 50 == 0:
        n = i + 1
        print(f"{n} rows {time.time()-t0:.0f}s  T={T} scanned: ub {T - tot_ub / n:.2f}  "
              f"g* {T - tot_skip / n:.2f}  both {T - tot_both / n:.2f}  "
              f"labels below g*: mean {np.mean(frac_lab):.3f} median {np.median(frac_lab):.3f}", flush=True)
