"""Heavy-row split parameters (split_rows M, pieces P): the whole-graph launch
(N = 1) and the slowest of the 8 work-balanced shards (the N = 8 step's hot
part), each the best of AB_REPS runs.  Results are identical for every (M, P)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-pathsim_amd"))
import torch
from dpathsim.synth import synth_config, CONFIGS
from dpathsim.engine import build_engine
from dpathsim.dist import balanced_bounds
import dpathsim

cfg = os.environ.get("AB_CONFIG", "config3")
K = CONFIGS[cfg][4]
t = synth_config(cfg).typed(dpathsim.METAPATHS[CONFIGS[cfg][3]])
eng = build_engine(t)
reps = int(os.environ.get("AB_REPS", "2"))
shards = balanced_bounds(eng.row_work(), 8)
eng.topk(K, 0, 20000)


def timed(r0, r1, M, P):
    best = 1e30
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(); eng.topk(K, r0, r1, split_rows=M, pieces=P); e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best


for M, P in [(256, 16), (128, 16), (512, 16), (1024, 16), (256, 32), (512, 32), (1024, 8), (2048, 8)]:
    full = timed(0, t.n_authors, M, P)
    sh = [timed(a, b, M, P) for a, b in shards]
    print(f"{cfg} M={M} P={P}: N=1 {full:.2f} ms, 8 shards max {max(sh):.2f} min {min(sh):.2f} ms", flush=True)
