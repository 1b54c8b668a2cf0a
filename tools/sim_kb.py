"""Simulation (CPU, numpy): tiles (and 16-byte chunks) the hot kernel scans per
row under per-tile bounds, including the g-budget (knapsack) bound.

Targets are relabelled by ascending g and cut into tiles of W labels (the
kernel's layout).  Tile t of row x is skipped when a bound B[x,t] on
max_{y in t} M[x,y] is below mneed(tau, gx + gmin_t).

  ub   sum_v a_v * maxc[v,t]                          (round-2 kernel)
  kb   max sum_v a_v b_v  s.t.  0 <= b_v <= maxc[v,t],  sum_v b_v s_v <= gmax_t
       (fractional knapsack, greedy by a_v / s_v):  every target y of tile t
       has g[y] = sum_u C[y,u] s_u >= sum_{v in x} C[y,v] s_v, and g[y] <= gmax_t
  kbs  the score form of kb: skip when max over budgets B in [0, gmax_t] of
       f(B) - tau/2 (gx + max(gmin_t, B)) < 0  (f = the knapsack value at B)
  cs   floor(sqrt(M[x,x] * max_{y in t} M[y,y]))
  min  min(ub, kb, cs)
each with the running tau (ascending and best-first tile orders) and with the
final tau; "perfect" = tiles holding a target that scores >= the final tau.
a_v = C[x,v], s_v = column sum of C (the global-walk weights).
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
s = s.astype(np.float64)
print(f"{cfg}: NA={NA} nnz={len(cc)} build {time.time()-t0:.1f}s", flush=True)
gg = gg[:NA].astype(np.int64)
C = sp.csr_matrix((cv.astype(np.int64), cc, cp), shape=(NA, NV))
CT = C.T.tocsr()
dg = np.asarray(C.multiply(C).sum(1)).ravel().astype(np.int64)
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
g_lab = gg[order]
gmin = g_lab[np.arange(T) * W].astype(np.float64)
gmax = g_lab[np.minimum(np.arange(T) * W + W - 1, NA - 1)].astype(np.float64)
print(f"tables {time.time()-t0:.1f}s", flush=True)

rng = np.random.default_rng(7)
rows = np.sort(rng.choice(NA, size=nrows, replace=False))


def knap(a, sv, mx):
    """Fractional knapsack per tile: value at budget gmax_t, plus the breakpoint
    table (budget, value) for the score form."""
    o = np.argsort(-(a / sv), kind="stable")
    rem = gmax.copy()
    val = np.zeros(T)
    bps_b = [np.zeros(T)]
    bps_v = [np.zeros(T)]
    used = np.zeros(T)
    for j in o:
        cap = mx[j].astype(np.float64) * sv[j]
        take = np.minimum(cap, rem)
        val += a[j] * take / sv[j]
        rem -= take
        used += take
        bps_b.append(used.copy())
        bps_v.append(val.copy())
    return val, np.array(bps_b), np.array(bps_v)


def kbs_ok(tau, tt, gx, bb, bv):
    """True if some budget B in [0, gmax_t] has f(B) >= tau/2 (gx + max(gmin_t, B))."""
    if tau <= 0:
        return True
    tt_ = tau * 0.5 * (1 - 2.0 ** -40)
    b, v = bb[:, tt], bv[:, tt]
    # candidate budgets: f's breakpoints and gmin_t (f linear between breakpoints)
    cand_b = np.concatenate([b, [min(gmin[tt], b[-1])]])
    cand_v = np.concatenate([v, [np.interp(min(gmin[tt], b[-1]), b, v)]])
    return bool(np.any(cand_v >= tt_ * (gx + np.maximum(gmin[tt], cand_b)) - 1e-9))


def scan(bound, tile_best, gx, order_t, tau_fixed=None, chunks=None, extra=None):
    best = np.full(k, -1.0)
    n = 0
    nch = 0
    for tt in order_t:
        tau = tau_fixed if tau_fixed is not None else best[k - 1]
        if bound[tt] <= 0:
            continue
        if tau > 0 and bound[tt] < np.ceil(tau * (gx + gmin[tt]) * 0.5 * (1 - 2.0 ** -40)):
            continue
        if extra is not None and not extra(tau, tt):
            continue
        n += 1
        nch += chunks[tt]
        best = -np.sort(-np.concatenate([best, tile_best[tt]]))[:k]
    return n, nch


keys = []
res = {}
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
        a = cv[b0:b1].astype(np.float64)
        mx = maxc[cc[b0:b1]]
        ub = (a[:, None] * mx).sum(0)
        kb, bb, bv = knap(a, s[cc[b0:b1]], mx)
        kb = np.floor(kb + 1e-9)
        cs = np.floor(np.sqrt(dg[x].astype(np.float64) * maxdg))
        mn = np.minimum(np.minimum(ub, kb), cs)
        allsc = np.sort(sc)[::-1]
        tau_final = allsc[k - 1] if len(allsc) >= k else -1.0
        chunks = ((bcnt[cc[b0:b1]] + 7) // 8).sum(0)
        asc = np.arange(T)
        bf = np.argsort(-(2.0 * mn / (gx + gmin)), kind="stable")
        ex = lambda tau, tt: kbs_ok(tau, tt, gx, bb, bv)  # noqa: E731
        runs = {
            "all": (np.ones(T), asc, None, None),
            "ub": (ub, asc, None, None),
            "ub_fin": (ub, asc, tau_final, None),
            "kb": (kb, asc, None, None),
            "kb_fin": (kb, asc, tau_final, None),
            "min": (mn, asc, None, None),
            "min_bf": (mn, bf, None, None),
            "min_fin": (mn, asc, tau_final, None),
            "kbs": (mn, asc, None, ex),
            "kbs_bf": (mn, bf, None, ex),
            "kbs_fin": (mn, asc, tau_final, ex),
            "perfect": (tmax, asc, tau_final, None),
        }
        for nm, (bd, ot, tf, extra) in runs.items():
            n, nch = scan(bd, tile_best, gx, ot, tau_fixed=tf, chunks=chunks, extra=extra)
            r0 = res.setdefault(nm, [0, 0])
            r0[0] += n
            r0[1] += nch
    nn = i0 + len(rr)
    print(f"{nn} rows {time.time()-tb0:.0f}s  tiles/row (chunks/row):", flush=True)
    print("  " + "  ".join(f"{kk}={v[0]/nn:.1f} ({v[1]/nn:.0f})" for kk, v in res.items()), flush=True)
