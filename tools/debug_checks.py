"""Round 6: the hot kernel's bucket check of the debug build (make debug,
DPATHSIM_LIB=.../libdpathsim_debug.so): run the full config3 top-k (the bench
launch: heavy rows split) and print the first failing lane's record from the
counter workspace (words 48..55: line, q, off, bj, base_j, pre_j, pre_n,
nq | (venue + 1) << 32), or that none failed."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-pathsim_amd"))
import torch

from dpathsim.engine import build_engine
from dpathsim.synth import synth_config

cfg = os.environ.get("DBG_CONFIG", "config3")
eng = build_engine(synth_config(cfg, scale=float(os.environ.get("DBG_SCALE", "1"))).typed())
for split in (0, None):
    eng.topk(10, split_rows=split)
    torch.cuda.synchronize()
    c = eng.tensor("topk_ws")[:512].view(torch.int64).cpu().tolist()
    names = ["line", "q", "off", "bj", "base_j", "pre_j", "pre_n", "nq|venue"]
    rec = dict(zip(names, c[48:56]))
    print(f"{cfg} split_rows={split}: " + ("no failed check" if c[48] == 0 else f"FAILED {rec} "
          f"(nq {c[55] & 0xFFFFFFFF}, venue {(c[55] >> 32) - 1})"), flush=True)
