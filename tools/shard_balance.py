"""Predict the multi-GPU step on one GPU: for world = 2, 4, 8, time the hot
kernel on every rank's shard (dpathsim.dist.balanced_bounds over row_work,
exactly what bench.py --gpus N runs per rank) and report max / mean shard
time, plus the build time every rank pays.  Prints JSON lines."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "distributed-pathsim_amd"))
import numpy as np
import torch

from dpathsim.dist import balanced_bounds
from dpathsim.engine import build_engine
from dpathsim.synth import synth_config

cfg = os.environ.get("SB_CONFIG", "config3")
k = int(os.environ.get("SB_K", "10"))
t = synth_config(cfg).typed()
eng = build_engine(t)
NA = t.n_authors


def timed(fn, reps=2):
    best = 1e30
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best


eng.topk(k, 0, 20000)
full = timed(lambda: eng.topk(k))
build = timed(lambda: eng.build(check=False))
print(json.dumps({"config": cfg, "world": 1, "hot_ms": full, "build_ms": build}), flush=True)
for world in (2, 4, 8):
    bounds = balanced_bounds(eng.row_work(), world)
    ms = [timed(lambda a=a, b=b: eng.topk(k, a, b)) for a, b in bounds]
    print(json.dumps({"config": cfg, "world": world, "shard_ms": [round(m, 2) for m in ms],
                      "max_ms": max(ms), "mean_ms": float(np.mean(ms)),
                      "imbalance": max(ms) / float(np.mean(ms)),
                      "predicted_step_ms": max(ms) + build,
                      "predicted_speedup": (full + build) / (max(ms) + build)}), flush=True)
