"""Hot-kernel timing on config3 (first R rows) across tile widths and ablations.

Results must be identical across tile widths (bit-exact); ablation runs
(DPATHSIM_ABLATE: 1 no LDS adds, 2 no candidate scoring, 4 no scatter) are
timing-only.
"""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-pathsim_amd"))
import numpy as np
import torch
from dpathsim.synth import synth_config
from dpathsim.engine import build_engine

R = int(os.environ.get("AB_ROWS", "200000"))
K = int(os.environ.get("AB_K", "10"))
Ws = [int(w) for w in os.environ.get("AB_W", "8192,16384").split(",")]
ablations = [a for a in os.environ.get("AB_ABLATE", "1,2,4").split(",") if a]
t = synth_config(os.environ.get("AB_CONFIG", "config3")).typed()
res = {}
ref = None


def timed(eng, rows):
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record(); o = eng.topk(K, 0, rows); e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1), o


for W in Ws:
    eng = build_engine(t, tile_w=W)
    os.environ["DPATHSIM_ABLATE"] = "0"
    eng.topk(K, 0, 20000); torch.cuda.synchronize()
    ms, o = timed(eng, R)
    o = [a.cpu().numpy() for a in o]
    res[f"W{W}"] = ms
    print(f"W={W}: {ms:.1f} ms for {R} rows", flush=True)
    if ref is None:
        ref = o
    else:
        bad = np.flatnonzero((o[0] != ref[0]).any(1) | (o[1] != ref[1]).any(1) |
                             (o[2].view(np.int64) != ref[2].view(np.int64)).any(1))
        print(f"  vs W={Ws[0]}: {len(bad)} rows differ {bad[:5].tolist()}", flush=True)
    for ab in ablations:
        os.environ["DPATHSIM_ABLATE"] = ab
        ms, _ = timed(eng, R)
        res[f"W{W}_ablate{ab}"] = ms
        print(f"  ablate {ab}: {ms:.1f} ms", flush=True)
        if ab == "16":   # shader-clock cycles per phase, summed over waves
            c = eng.tensor("topk_ws")[:256].view(torch.int64).cpu().tolist()
            names = ["scatter", "flush", "barrier1", "find", "prefetch", "epilogue", "barrier2"]
            st = max(c[15], 1)
            print("  cycles per wave-stage: " + " ".join(f"{n} {c[8 + i] / st:.0f}"
                                                         for i, n in enumerate(names))
                  + f" (stages {c[15]}, {c[15] / R:.1f} per row)", flush=True)
    os.environ["DPATHSIM_ABLATE"] = "8"
    timed(eng, R)
    c = eng.tensor("topk_ws")[:256].view(torch.int64).cpu().tolist()
    print(f"  counters per row: flushes {c[1]/R:.1f} candidates {c[2]/R:.1f} passers {c[3]/R:.1f} "
          f"tiles visited {c[4]/R:.1f} scanned {c[5]/R:.1f}", flush=True)
    nw = 1 if W <= 8192 else (8 if W == 65536 else 4)   # waves per row (dps_cct_topk)
    c[5] = c[5] or 1
    print(f"  per wave-stage: epilogue iterations {c[16]/(c[5]*nw):.2f} prefilter passes {c[17]/(c[5]*nw):.2f} "
          f"exact passes {c[18]/(c[5]*nw):.2f} extraction rounds {c[19]/(c[5]*nw):.2f} "
          f"fast loads {c[20]/(c[5]*nw):.2f} slow loads {c[21]/(c[5]*nw):.2f}", flush=True)
    os.environ["DPATHSIM_ABLATE"] = "0"
print(json.dumps(res))
