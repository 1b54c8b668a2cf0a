"""A/B of the hot kernel: general k_cct_topk (DPATHSIM_LEAN=0) vs the lean
one-wave kernel k_cct1 (default at W = 8192) on a synthetic config, full
launch as bench.py runs it (heaviest rows first, split heavy rows).  The two
outputs must be identical bit for bit."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-pathsim_amd"))
import numpy as np
import torch
from dpathsim.synth import synth_config
from dpathsim.engine import build_engine

cfg = os.environ.get("AB_CONFIG", "config3")
k = int(os.environ.get("AB_K", "10"))
R = int(os.environ.get("AB_ROWS", "0"))
reps = int(os.environ.get("AB_REPS", "3"))
eng = build_engine(synth_config(cfg).typed(), tile_w=8192)
NA = eng.typed.n_authors
R = NA if R <= 0 else min(R, NA)
res = {}
for mode in os.environ.get("AB_MODES", "0,1").split(","):
    if mode.startswith("w"):   # lean kernel, waves per CU
        os.environ["DPATHSIM_LEAN_WPC"] = mode[1:]; os.environ["DPATHSIM_LEAN"] = "1"
    else:
        os.environ["DPATHSIM_LEAN"] = mode
    eng.topk(k, 0, min(R, 20000)); torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(); o = eng.topk(k, 0, R); e1.record(); torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    res[mode] = [t.cpu().numpy() for t in o]
    print(f"{cfg} k={k} rows={R} lean={mode}: {best:.2f} ms", flush=True)
if "0" in res and "1" in res:
    a, b = res["0"], res["1"]
    bad = np.flatnonzero((a[0] != b[0]).any(1) | (a[1] != b[1]).any(1) |
                         (a[2].view(np.int64) != b[2].view(np.int64)).any(1))
    print(f"rows differing lean vs general: {len(bad)} {bad[:8].tolist()}", flush=True)
    if len(bad):
        i = bad[0]
        print("general", a[0][i], a[1][i], "\nlean   ", b[0][i], b[1][i], flush=True)
        sys.exit(1)
