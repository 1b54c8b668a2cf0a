"""One device build of AB_CONFIG (after two warm-up builds), for a rocprofv3
--kernel-trace run: tools/build_trace_summary.py then lists the kernels of
the last build in launch order with their durations, per build phase."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "distributed-pathsim_amd"))
import torch

from dpathsim.engine import PathSimEngine
from dpathsim.graph import METAPATHS
from dpathsim.synth import CONFIGS, synth_config

cfg = os.environ.get("AB_CONFIG", "config3")
t = synth_config(cfg).typed(METAPATHS[CONFIGS[cfg][3]])
eng = PathSimEngine(t, tile_w=int(os.environ.get("AB_W", "16384"))).upload()
for _ in range(3):
    eng.build(check=False)
    torch.cuda.synchronize()
print("done", cfg, flush=True)
