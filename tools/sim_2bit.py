"""Simulation (CPU, numpy; round 6): would 2-bit counters over 32768-target
tiles (the same 8 KiB accumulator) save passes?  A 32768-wide super-tile whose
bound sum_v C[x,v] * maxc32[v,T] is at most 3 could run as ONE 2-bit pass
instead of its two 16384-target tiles' passes (1 each at a 4-bit bound <= 15,
else 2 u8 halves).  Counts passes per row without tau pruning on a sample of
config3 rows."""
import os, sys, time
import numpy as np, scipy.sparse as sp
sys.path.insert(0, "/root/repo/distributed-pathsim_amd"); sys.path.insert(0, "/root/repo/oracle")
from dpathsim.synth import synth_config
import pathsim_oracle as po
t0=time.time()
g = synth_config("config3"); t = g.typed(); co = po.COracle.from_typed(t)
cp, cc, cv, s, gg = co.export()
NA, NV = t.n_authors, t.n_mids
cp = cp[:NA+1]; cc = cc[:cp[-1]]; cv = cv[:cp[-1]]
gg = gg[:NA].astype(np.int64)
order = np.argsort(gg, kind="stable"); rank = np.empty(NA, np.int64); rank[order] = np.arange(NA)
row_of = np.repeat(np.arange(NA), np.diff(cp))
res = {}
for W in (16384, 32768):
    T = (NA + W - 1)//W
    maxc = np.zeros((NV, T), np.int64)
    np.maximum.at(maxc, (cc, rank[row_of]//W), cv)
    res[W] = maxc
print("built", time.time()-t0, flush=True)
rng = np.random.default_rng(3); rows = rng.choice(NA, 3000, replace=False)
m16, m32 = res[16384], res[32768]
tot16 = 0; pass16 = 0; pass_new = 0
for x in rows:
    b0, b1 = cp[x], cp[x+1]
    c = cv[b0:b1].astype(np.int64); v = cc[b0:b1]
    ub16 = (c[:, None] * m16[v]).sum(0)          # per 16384 tile
    ub32 = (c[:, None] * m32[v]).sum(0)
    # current passes (no tau pruning): tile with ub16 > 0: 1 pass if <= 15, else 2 (u8 halves), ignoring wide
    p16 = np.where(ub16 == 0, 0, np.where(ub16 <= 15, 1, 2))
    pass16 += p16.sum()
    # new: super-tile with ub32 <= 3 and > 0: one 2-bit pass replaces its two 16384 tiles' passes
    T32 = len(ub32)
    pn = 0
    for T_ in range(T32):
        a = p16[2*T_: 2*T_+2].sum()
        if ub32[T_] == 0: continue
        pn += 1 if ub32[T_] <= 3 else a
    pass_new += pn
print(f"rows {len(rows)}: passes (no pruning) 16384-scheme {pass16/len(rows):.1f}/row, with 2-bit 32768 passes {pass_new/len(rows):.1f}/row ({1-pass_new/pass16:.3f} fewer)")
