"""A/B one library build: hot-kernel time on config3 rows [0, R) + output digest.

DPATHSIM_LIB selects the library; AB_TAG names the line.  Digests must agree
across builds (the outputs are exact).
"""
import hashlib, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-pathsim_amd"))
import torch
from dpathsim.synth import synth_config
from dpathsim.engine import build_engine

R = int(os.environ.get("AB_ROWS", "1000000"))
cfg = os.environ.get("AB_CONFIG", "config3")
k = int(os.environ.get("AB_K", "10"))
eng = build_engine(synth_config(cfg).typed(), tile_w=int(os.environ.get("AB_W", "32768")))
R = min(R, eng.typed.n_authors)
eng.topk(k, 0, 20000); torch.cuda.synchronize()
best = 1e30
for _ in range(int(os.environ.get("AB_REPS", "2"))):
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record(); o = eng.topk(k, 0, R); e1.record(); torch.cuda.synchronize()
    best = min(best, e0.elapsed_time(e1))
h = hashlib.md5()
for t in o:
    h.update(t.cpu().numpy().tobytes())
print(f"{os.environ.get('AB_TAG', 'lib')}: {cfg} rows {R} k {k}: {best:.1f} ms  digest {h.hexdigest()}", flush=True)
