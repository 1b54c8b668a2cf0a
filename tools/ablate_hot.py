import os, sys, time, json
sys.path.insert(0, 'distributed-pathsim_amd')
import torch
from dpathsim.synth import synth_config
from dpathsim.engine import build_engine
g = synth_config("config3"); t = g.typed()
res = {}
for W in (4096, 2048, 1024):
    eng = build_engine(t, tile_w=W)
    for mode in (0, 1, 2, 3, 4, 6):
        os.environ["DPATHSIM_ABLATE"] = str(mode)
        eng.topk(10, 0, 50000); torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(); eng.topk(10, 0, 200000); e1.record(); torch.cuda.synchronize()
        res[f"W{W}_mode{mode}"] = e0.elapsed_time(e1)
        print(W, mode, res[f"W{W}_mode{mode}"], flush=True)
    os.environ["DPATHSIM_ABLATE"] = "0"
print(json.dumps(res))
