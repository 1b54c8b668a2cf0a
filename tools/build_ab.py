"""Device build phases on config3 (or AB_CONFIG) under several env settings.

AB_ENV="DPATHSIM_TILE_LPB=1024;DPATHSIM_TILE_LPB=4096" -> one line per setting
with the median phase times (ms) of AB_REPS timed builds, the median untimed
build wall time (host enqueue + device, one sync) and the row_work + argsort
time.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "distributed-pathsim_amd"))
import numpy as np
import torch

from dpathsim.engine import PathSimEngine
from dpathsim.synth import synth_config

from dpathsim.graph import METAPATHS
from dpathsim.synth import CONFIGS

_cfg = os.environ.get("AB_CONFIG", "config3")
t = synth_config(_cfg).typed(METAPATHS[CONFIGS[_cfg][3]])
reps = int(os.environ.get("AB_REPS", "5"))
eng = PathSimEngine(t, tile_w=int(os.environ.get("AB_W", "8192"))).upload()
for setting in os.environ.get("AB_ENV", "").split(";"):
    env = dict(kv.split("=", 1) for kv in setting.split(",") if kv)
    os.environ.update(env)
    eng.build()
    phases = []
    for _ in range(reps):
        eng.build(timed=True)
        phases.append(dict(eng.info.phase_ms))
    walls = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.build(check=False)
        w = eng.row_work()
        order = torch.argsort(w, descending=True, stable=True)
        torch.cuda.synchronize()
        walls.append((time.perf_counter() - t0) * 1e3)
    # host enqueue time of one build (no sync inside): below the device time
    # the GPU never waits for the host, so a graph capture would not shorten it
    enq = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.build(check=False)
        enq.append((time.perf_counter() - t0) * 1e3)
        torch.cuda.synchronize()
    med = {k: float(np.median([p[k] for p in phases])) for k in phases[0]}
    print(json.dumps({"env": env, "phase_ms": med, "phase_total_ms": sum(med.values()),
                      "build_plus_plan_wall_ms": float(np.median(walls)),
                      "host_enqueue_ms": float(np.median(enq))}), flush=True)
    for k in env:
        os.environ.pop(k)
