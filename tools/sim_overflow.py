"""Simulation (CPU, numpy): how often a 16384-target tile whose 4-bit bound
exceeds 15 really holds a count of 16 or more (the optimistic 4-bit passes of
dps_cct1.hip, kOptMax).

For a row sample stratified by row work (sum_{v in x} n_v), with the row's
final tau: the live tiles (bound >= mneed(tau, gx + gmin_t)), those whose 4-bit
bound exceeds 15 (the kernel used to split them into two u8 halves), and among
those the tiles -- and 8192-target halves -- whose largest M[x,y] reaches 16
(an optimistic pass overflows there and the half runs again).
  python tools/sim_overflow.py [config] [k] [rows per band]
"""
import os
import sys

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "distributed-pathsim_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
from dpathsim.synth import synth_config  # noqa: E402
import pathsim_oracle as po  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "config3"
k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
nrows = int(sys.argv[3]) if len(sys.argv) > 3 else 40
W = 16384
t = synth_config(cfg).typed()
co = po.COracle.from_typed(t)
cp, cc, cv, s, gg = co.export()
NA, NV = t.n_authors, t.n_mids
cp = cp[: NA + 1]
cc = cc[: cp[-1]]
cv = cv[: cp[-1]].astype(np.int64)
gg = gg[:NA].astype(np.int64)
C = sp.csr_matrix((cv, cc, cp), shape=(NA, NV))
order = np.argsort(gg, kind="stable")
rank = np.empty(NA, np.int64)
rank[order] = np.arange(NA)
T = (NA + W - 1) // W
g_lab = gg[order]
gmin = g_lab[np.arange(T) * W]
row_of = np.repeat(np.arange(NA), np.diff(cp))
tl = rank // W
maxc = np.zeros((NV, T), np.int64)
np.maximum.at(maxc, (cc, tl[row_of]), cv)
T8 = (NA + W // 2 - 1) // (W // 2)
maxh = np.zeros((NV, T8), np.int64)
np.maximum.at(maxh, (cc, (rank // (W // 2))[row_of]), cv)
n_v = np.bincount(cc, minlength=NV)
deg = np.diff(cp)
terms = np.add.reduceat(n_v[cc], cp[:-1]) * (deg > 0)
rng = np.random.default_rng(9)
qs = np.quantile(terms, [0, 0.33, 0.66, 0.9, 1.0])
for band in range(4):
    pool = np.flatnonzero((terms >= qs[band]) & (terms <= qs[band + 1]) & (deg > 0))
    rows = rng.choice(pool, min(nrows, len(pool)), replace=False)
    live = split = ovf = ovf_h = both15 = chk_h = 0
    n = 0
    for x in rows:
        a0, a1 = cp[x], cp[x + 1]
        v, a = cc[a0:a1], cv[a0:a1]
        mrow = np.asarray(C @ sp.csr_matrix((a, v, [0, len(v)]), shape=(1, NV)).T.todense()).ravel()
        mrow[x] = 0
        sc = 2.0 * mrow / (gg[x] + gg)
        tau = np.sort(sc)[-k]
        if tau <= 0:
            continue
        n += 1
        ub = (a[:, None] * maxc[v]).sum(0)
        mneed = np.ceil(tau * (gg[x] + gmin) / 2.0 - 1e-9)
        lv = ub >= mneed
        mt = np.zeros(T, np.int64)
        np.maximum.at(mt, tl, mrow)
        mh = np.zeros(2 * T, np.int64)
        np.maximum.at(mh, rank // (W // 2), mrow)
        sp_t = lv & (ub > 15)
        uh = (a[:, None] * maxh[v]).sum(0)
        uh = np.pad(uh, (0, 2 * T - len(uh)))
        ha, hb2 = uh[0::2], uh[1::2]
        both15 += (sp_t & (ha <= 15) & (hb2 <= 15)).sum()
        chk_h += (sp_t & (ha > 15)).sum() + (sp_t & (hb2 > 15)).sum()
        live += lv.sum()
        split += sp_t.sum()
        ovf += (sp_t & (mt >= 16)).sum()
        ovf_h += (np.repeat(sp_t, 2)[: len(mh)] & (mh >= 16)).sum()
    print(f"{cfg} band {band} (row work {qs[band]:.0f}..{qs[band + 1]:.0f}), {n} rows: live tiles/row "
          f"{live / n:.1f}, bound > 15: {split / n:.1f}, of which a count >= 16: {ovf / n:.2f} tiles "
          f"({ovf_h / n:.2f} halves); both half bounds <= 15: {both15 / n:.1f} tiles; halves with a "
          f"bound > 15 (to check): {chk_h / n:.1f}", flush=True)
