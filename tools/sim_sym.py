"""Simulation (CPU): exploit M's symmetry in the hot kernel.

Targets are relabelled by ascending g and tiled (W labels per tile).  Row x
scans only tiles >= tile(x) - B (its band and everything above); a pair (x, y)
with tile(y) > tile(x) + B is then seen only by x, which must hand it to y
("emission") when it can enter y's top-k: score >= tau_y.  Reported:
  work      sum over rows of the C^T entries scanned, as a share of the full scan
  tiles     tiles scanned per row (passes), as a share of T
  emit      per row: pairs with score >= tau_full[y] (the minimum any valid
            threshold must emit) and epilogue candidates under a per-2048-target
            block threshold mneed(min tau over the block, gx + min g of the block)
usage: sim_sym.py [config] [B] [sample rows]
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
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
nsamp = int(sys.argv[3]) if len(sys.argv) > 3 else 400
W = int(os.environ.get("SIM_W", "16384"))
k = 10
t0 = time.time()
t = synth_config(cfg).typed()
co = po.COracle.from_typed(t)
cp, cc, cv, s, g = co.export()
NA, NV = t.n_authors, t.n_mids
print(f"{cfg}: NA={NA} nnz={len(cc)} build {time.time() - t0:.1f}s", flush=True)
tau_path = f"/tmp/sim_sym_tau_{cfg}.npy"
if os.path.exists(tau_path):
    tau = np.load(tau_path)
else:
    t1 = time.time()
    _, _, sc = co.topk(k, 0, NA)
    tau = sc[:, k - 1].copy()
    np.save(tau_path, tau)
    print(f"oracle top-{k} of all rows {time.time() - t1:.1f}s", flush=True)
order = np.argsort(g, kind="stable")
lab = np.empty(NA, np.int64)
lab[order] = np.arange(NA)
tile = lab // W
T = int(tile.max()) + 1
row = np.repeat(np.arange(NA), np.diff(cp))
# members of each venue by label: key = v * 2^21 + label
key = np.sort(cc.astype(np.int64) * (1 << 21) + lab[row])
n_v = np.bincount(cc, minlength=NV)
lo = np.maximum(tile[row] - B, 0) * W
pos = np.searchsorted(key, cc.astype(np.int64) * (1 << 21) + lo)
end = np.searchsorted(key, cc.astype(np.int64) * (1 << 21) + (1 << 21))
scanned = (end - pos).sum()
full = n_v[cc].sum()
tiles = (T - np.maximum(tile - B, 0)).sum()
print(f"B={B} W={W} T={T}: work {scanned / full:.3f} of the full scan, "
      f"tiles per row {tiles / NA:.1f} of {T} ({tiles / NA / T:.3f})", flush=True)
# work share by tile of the row (where the remaining work sits)
wt = np.bincount(tile[row], weights=(end - pos).astype(np.float64), minlength=T)
wf = np.bincount(tile[row], weights=n_v[cc].astype(np.float64), minlength=T)
print("  remaining work share by row tile (first 8, last 8):",
      " ".join(f"{x:.3f}" for x in (wt / wt.sum())[:8]), "...",
      " ".join(f"{x:.3f}" for x in (wt / wt.sum())[-8:]), flush=True)
print("  full work share by row tile (last 8):", " ".join(f"{x:.3f}" for x in (wf / wf.sum())[-8:]))
# emissions on a row sample
C = sp.csr_matrix((cv.astype(np.float64), cc, cp), shape=(NA, NV))
blk = lab // 2048
nb = int(blk.max()) + 1
tau_b = np.full(nb, np.inf)
np.minimum.at(tau_b, blk, tau)
g_b = np.full(nb, np.inf)
np.minimum.at(g_b, blk, g.astype(np.float64))
rng = np.random.default_rng(1)
xs = rng.choice(NA, nsamp, replace=False)
# variant: labels re-sorted by tau inside each tile (tile membership kept)
lab2 = np.empty(NA, np.int64)
SG = int(os.environ.get("SIM_SORT_GROUP", str(W)))
o2 = np.lexsort((tau, lab // SG))                # by label group, then tau ascending
lab2[o2] = np.arange(NA)
blk2 = lab2 // 2048
nb2 = int(blk2.max()) + 1
tau_b2 = np.full(nb2, np.inf)
np.minimum.at(tau_b2, blk2, tau)
g_b2 = np.full(nb2, np.inf)
np.minimum.at(g_b2, blk2, g.astype(np.float64))
tg_b2 = np.full(nb2, np.inf)
np.minimum.at(tg_b2, blk2, tau * g)
# variant 3: 8-label groups (whole accumulator dwords) re-sorted by their
# smallest tau inside each 8192-label half tile (what a relabel pass over the
# built tiles can do: l % 8 and the half tile are kept)
grp = lab // 8
ng = int(grp.max()) + 1
gt = np.full(ng, np.inf)
np.minimum.at(gt, grp, tau)
half = np.arange(ng) // 1024                      # 1024 groups of 8 per 8192 labels
og = np.lexsort((gt, half))                       # new group order
newpos = np.empty(ng, np.int64)
newpos[og] = np.arange(ng)
lab3 = newpos[grp] * 8 + lab % 8
blk3 = lab3 // 2048
tau_b3 = np.full(nb2, np.inf)
np.minimum.at(tau_b3, blk3, tau)
g_b3 = np.full(nb2, np.inf)
np.minimum.at(g_b3, blk3, g.astype(np.float64))
e_c3 = x3 = 0
# variant 4: the rows below the q-quantile of tau in each 2048-label block scan
# every tile themselves (no records), so the block threshold is that quantile
QS = (0.1, 0.25, 0.5)
tq = {}
for q in QS:
    tb = np.full(nb, np.inf)
    srt = np.lexsort((tau, blk))
    bs = np.bincount(blk, minlength=nb)
    st0 = np.concatenate([[0], np.cumsum(bs)[:-1]])
    qi = st0 + np.floor(q * bs).astype(np.int64)
    tb = tau[srt[np.minimum(qi, len(srt) - 1)]]
    weak = tau < tb[blk]
    extra = ((n_v[cc] - (end - pos)) * weak[row]).sum() / full
    tq[q] = (tb, weak, extra)
e_q = {q: 0 for q in QS}
e_c2 = e_c2b = 0
x1 = x2 = 0
g32 = lab // 32
n32 = int(g32.max()) + 1
tau_32 = np.full(n32, np.inf)
np.minimum.at(tau_32, g32, tau)
g_32 = np.full(n32, np.inf)
np.minimum.at(g_32, g32, g.astype(np.float64))
e_true = e_cand = e_c32 = e_exact = 0
t1 = time.time()
for x in xs:
    M = C @ C.getrow(x).T.toarray().ravel()
    far = tile > tile[x] + B
    sc = 2 * M / (g[x] + g)
    e_true += int(((sc >= tau) & far & (M > 0)).sum())
    m_need = np.ceil(tau_b[blk] * (g[x] + g_b[blk]) / 2)
    e_cand += int(((M >= np.maximum(m_need, 1)) & far).sum())
    m32 = np.ceil(tau_32[g32] * (g[x] + g_32[g32]) / 2)
    e_c32 += int(((M >= np.maximum(m32, 1)) & far).sum())
    m2 = np.ceil(tau_b2[blk2] * (g[x] + g_b2[blk2]) / 2)
    e_c2 += int(((M >= np.maximum(m2, 1)) & far).sum())
    m2b = np.ceil((tau_b2[blk2] * g[x] + tg_b2[blk2]) / 2)
    e_c2b += int(((M >= np.maximum(m2b, 1)) & far).sum())
    own = tile >= tile[x] - B
    mx1 = np.ceil(tau[x] * (g[x] + g_b[blk]) / 2)
    x1 += int(((M >= np.maximum(mx1, 1)) & own).sum())
    mx2 = np.ceil(tau[x] * (g[x] + g_b2[blk2]) / 2)
    x2 += int(((M >= np.maximum(mx2, 1)) & own).sum())
    m3 = np.ceil(tau_b3[blk3] * (g[x] + g_b3[blk3]) / 2)
    e_c3 += int(((M >= np.maximum(m3, 1)) & far).sum())
    mx3 = np.ceil(tau[x] * (g[x] + g_b3[blk3]) / 2)
    x3 += int(((M >= np.maximum(mx3, 1)) & own).sum())
    for q in QS:
        tb, weak, _ = tq[q]
        mq = np.ceil(tb[blk] * (g[x] + g_b[blk]) / 2)
        e_q[q] += int(((M >= np.maximum(mq, 1)) & far & ~weak).sum())
    mex = np.ceil(tau * (g[x] + g) / 2)
    e_exact += int(((M >= np.maximum(mex, 1)) & far).sum())
print(f"emissions per row (sample {nsamp}, {time.time() - t1:.0f}s): true {e_true / nsamp:.2f}, "
      f"candidates: 2048-block threshold {e_cand / nsamp:.1f}, 32-group {e_c32 / nsamp:.1f}, "
      f"per-target {e_exact / nsamp:.1f}; tau-sorted tiles: 2048-block {e_c2 / nsamp:.1f}, "
      f"with min(tau*g) {e_c2b / nsamp:.1f}; x-side candidates (final tau, own tiles): "
      f"g-sorted {x1 / nsamp:.1f}, tau-sorted {x2 / nsamp:.1f}; 8-groups by tau in halves: "
      f"y-side {e_c3 / nsamp:.1f}, x-side {x3 / nsamp:.1f}", flush=True)
for q in QS:
    print(f"  weak below the {q:.2f} quantile per block: y-side {e_q[q] / nsamp:.1f}, "
          f"extra work {tq[q][2]:.3f} of the full scan", flush=True)
