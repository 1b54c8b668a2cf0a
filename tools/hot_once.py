"""Run the hot kernel once on config3 rows [0, R) (for rocprofv3 --pmc passes)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-pathsim_amd"))
import torch
from dpathsim.synth import synth_config
from dpathsim.engine import build_engine
from dpathsim import _lib
for kv in filter(None, os.environ.get("AB_TUNE", "").split(",")):   # "key=value,..."
    _lib.call("dps_set_tuning", *(int(v) for v in kv.split("=")))

R = int(os.environ.get("HOT_ROWS", "100000"))
W = int(os.environ.get("HOT_W", "16384"))
eng = build_engine(synth_config(os.environ.get("HOT_CONFIG", "config3")).typed(), tile_w=W,
                   venue_skip=os.environ.get("HOT_VS", "1" if W == 16384 else "0") == "1")
torch.cuda.synchronize()
eng.topk(10, 0, R)
torch.cuda.synchronize()
print("done", R, flush=True)
