"""Hot launch over all rows with and without the heavy-row split (results
identical): is the split worth its piece and merge overhead at N = 1?"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-pathsim_amd"))
import numpy as np
import torch
from dpathsim.synth import synth_config, CONFIGS
from dpathsim.engine import build_engine
import dpathsim

cfg = os.environ.get("AB_CONFIG", "config3")
K = CONFIGS[cfg][4]
t = synth_config(cfg).typed(dpathsim.METAPATHS[CONFIGS[cfg][3]])
eng = build_engine(t)
NA = t.n_authors
times = {0: [], None: []}
outs = {}
eng.topk(K, 0, 20000)
for rep in range(int(os.environ.get("AB_REPS", "3"))):
    for sr in (None, 0):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(); o = eng.topk(K, split_rows=sr); e1.record(); torch.cuda.synchronize()
        times[sr].append(e0.elapsed_time(e1))
        outs[sr] = [a.cpu().numpy() for a in o]
same = all(np.array_equal(a.view(np.int64) if a.dtype == np.float64 else a,
                          b.view(np.int64) if b.dtype == np.float64 else b)
           for a, b in zip(outs[None], outs[0]))
print(f"{cfg}: split {min(times[None]):.2f} ms, no split {min(times[0]):.2f} ms, identical {same}", flush=True)
