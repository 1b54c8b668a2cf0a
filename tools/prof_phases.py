"""Per-phase shader-clock breakdown of the hot kernel (DPATHSIM_ABLATE=16) on config3.

Prints, per wave-stage, the average cycles spent in: scatter (loads + LDS adds
issued), barrier 1, find next stage + prefetch, epilogue, barrier 2 (single
buffer only), flush; plus the plain kernel time for reference.
"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-pathsim_amd"))
import torch
from dpathsim.synth import synth_config
from dpathsim.engine import build_engine

R = int(os.environ.get("AB_ROWS", "200000"))
t = synth_config(os.environ.get("AB_CONFIG", "config3")).typed()
for W in [int(w) for w in os.environ.get("AB_W", "16384,32768").split(",")]:
    eng = build_engine(t, tile_w=W)
    os.environ["DPATHSIM_ABLATE"] = "0"
    eng.topk(10, 0, 20000); torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record(); eng.topk(10, 0, R); e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    os.environ["DPATHSIM_ABLATE"] = "16"
    e0.record(); eng.topk(10, 0, R); e1.record(); torch.cuda.synchronize()
    ms16 = e0.elapsed_time(e1)
    c = eng.tensor("topk_ws")[:256].view(torch.int64).cpu().tolist()
    os.environ["DPATHSIM_ABLATE"] = "0"
    nw = 1 if W <= 8192 else (8 if W == 65536 else 4)   # waves per row (dps_cct_topk)
    stages = c[15] / nw
    names = os.environ.get("PH_NAMES", "scatter,flush,barrier1,find,prefetch,epilogue,barrier2").split(",")
    tot = sum(c[8:8 + len(names)])
    print(f"W={W}: {ms:.1f} ms ({ms16:.1f} ms instrumented) for {R} rows; stages/row {stages / R:.1f}")
    for i, nm in enumerate(names):
        print(f"   {nm:14s} {c[8 + i] / c[15]:9.0f} cycles/wave-stage  {c[8 + i] / tot * 100:5.1f} %")
