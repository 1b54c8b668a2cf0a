"""Simulation (CPU, numpy): how many C^T entries a witness-pruned top-k scan reads.

For every source row x with true k-th score tau_x (from the C oracle), a target
y can reach tau_x only if some shared venue v "witnesses" it:
    2 a_v c_yv >= tau (w_v gx + c_yv s_v),   sum_v w_v <= 1   (mediant bound)
so with C^T buckets sorted by c descending only the prefix c_yv >= c_min(x,v)
must be read.  Prints the entries read per row for several weightings w.
"""
import sys, os, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "distributed-pathsim_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
from dpathsim.synth import synth_config
import pathsim_oracle as po

cfg = sys.argv[1] if len(sys.argv) > 1 else "config3_100k"
k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
nrows = int(sys.argv[3]) if len(sys.argv) > 3 else 20000
t0 = time.time()
g = synth_config(cfg)
t = g.typed()
co = po.COracle.from_typed(t)
cp, cc, cv, s, gg = co.export()
NA, NV = t.n_authors, t.n_mids
print(f"{cfg}: NA={NA} nnz={len(cc)} build {time.time()-t0:.1f}s", flush=True)
rng = np.random.default_rng(1)
rows = np.sort(rng.choice(NA, size=min(nrows, NA), replace=False))
t0 = time.time()
# oracle topk per sampled row (contiguous blocks would be faster; sample anyway)
taus = np.zeros(len(rows))
for i0 in range(0, len(rows), 1):
    pass
idx, cnt, sc = co.topk(k, 0, NA, threads=8) if NA <= 200_000 else (None, None, None)
if sc is None:
    # full config: compute only for sampled rows, one at a time in blocks
    sc_rows = []
    for r in rows:
        _, _, s1 = co.topk(k, int(r), int(r) + 1, threads=1)
        sc_rows.append(s1[0])
    sc_s = np.array(sc_rows)
else:
    sc_s = sc[rows]
tau = sc_s[:, k - 1]
print(f"oracle topk {time.time()-t0:.1f}s; tau median {np.median(tau):.3g}", flush=True)

rowlen = np.diff(cp)
row_of = np.repeat(np.arange(NA), rowlen)
n_v = np.bincount(cc, minlength=NV)
maxc = int(cv.max())
# cnt_ge[v, c] = members of venue v with c_yv >= c
hist = np.zeros((NV, maxc + 2), np.int64)
np.add.at(hist, (cc, cv), 1)
cnt_ge = np.cumsum(hist[:, ::-1], axis=1)[:, ::-1]

full = 0
res = {}
schemes = ["none", "uniform", "n_v", "heaviest", "s_v"]
for sch in schemes:
    res[sch] = 0
res["lightonly"] = 0
for i, x in enumerate(rows):
    b, e = cp[x], cp[x + 1]
    vs, a = cc[b:e], cv[b:e].astype(np.float64)
    full += n_v[vs].sum()
    tt = tau[i] * (1 - 2.0 ** -40)
    gx = float(gg[x])
    sv = s[vs].astype(np.float64)
    for sch in schemes:
        if sch == "none":
            w = np.zeros(len(vs))
        elif sch == "uniform":
            w = np.full(len(vs), 1.0 / len(vs))
        elif sch == "n_v":
            w = n_v[vs] / n_v[vs].sum()
        elif sch == "heaviest":
            w = np.zeros(len(vs)); w[np.argmax(n_v[vs])] = 1.0
        else:
            w = sv / sv.sum()
        if tt <= 0:
            res[sch] += n_v[vs].sum()
            continue
        den = 2 * a - tt * sv
        ok = den > 0
        cmin = np.full(len(vs), maxc + 1, np.int64)
        with np.errstate(divide="ignore", invalid="ignore"):
            cm = np.ceil(tt * w * gx / np.where(ok, den, 1.0))
        cmin[ok] = np.clip(cm[ok], 1, maxc + 1).astype(np.int64)
        res[sch] += cnt_ge[vs, cmin].sum()
print(f"rows {len(rows)}: full entries/row {full/len(rows):.0f}")
for sch in schemes:
    print(f"  {sch:10s} entries/row {res[sch]/len(rows):10.1f}  ({res[sch]/full:.4f} of full)")

# ---- tile-aware bound: targets relabelled by ascending g, tiles of W labels;
# gx + gy >= gx + lam*gmin_t + (1-lam)*gy_S, per (x, t) the best lam.
W = int(os.environ.get("SIM_W", "16384"))
order = np.argsort(gg, kind="stable")
rank = np.empty(NA, np.int64); rank[order] = np.arange(NA)
T = (NA + W - 1) // W
tile_of = rank[row_of] // W
gmin = gg[order][np.arange(T) * W].astype(np.float64)
hist3 = np.zeros((NV, T, maxc + 2), np.int32)
np.add.at(hist3, (cc, tile_of, cv), 1)
cge3 = np.cumsum(hist3[:, :, ::-1], axis=2)[:, :, ::-1]
tot = {lam: 0 for lam in (0.0, 0.5, 0.9, 1.0)}
best = 0
for i, x in enumerate(rows):
    b, e = cp[x], cp[x + 1]
    vs, a = cc[b:e], cv[b:e].astype(np.float64)
    tt = tau[i] * (1 - 2.0 ** -40)
    gx = float(gg[x]); sv = s[vs].astype(np.float64)
    w = n_v[vs] / n_v[vs].sum()
    per = []
    for lam in tot:
        if tt <= 0:
            c = np.full((len(vs), T), 1)
        else:
            den = 2 * a - tt * (1 - lam) * sv                     # [d]
            num = tt * w[:, None] * (gx + lam * gmin[None, :])     # [d, T]
            with np.errstate(divide="ignore", invalid="ignore"):
                c = np.ceil(num / np.where(den > 0, den, 1.0)[:, None])
            c = np.where(den[:, None] > 0, np.clip(c, 1, maxc + 1), maxc + 1).astype(np.int64)
        n = cge3[vs[:, None], np.arange(T)[None, :], c]             # [d, T]
        tot[lam] += n.sum()
        per.append(n.sum(0))
    best += np.min(np.array(per), axis=0).sum()
print(f"tile-aware (W={W}, T={T}):")
for lam in tot:
    print(f"  lam={lam:.1f} entries/row {tot[lam]/len(rows):10.1f} ({tot[lam]/full:.4f})")
print(f"  best lam per (x,t) {best/len(rows):10.1f} ({best/full:.4f})")
