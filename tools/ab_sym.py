"""A/B of the symmetric mode on a config (all rows, bench shape): plain launch
(venue skipping on and off) against dps_cct_sym; times (best of AB_REPS, events
around eng.topk), kernel counts, records, and bit-identity of the outputs."""
import hashlib
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-pathsim_amd"))
import numpy as np
import torch
from dpathsim.engine import build_engine
from dpathsim.synth import synth_config, CONFIGS
import dpathsim

cfg = os.environ.get("AB_CONFIG", "config3")
W = int(os.environ.get("AB_W", "16384"))
K = int(os.environ.get("AB_K", str(CONFIGS[cfg][4])))
reps = int(os.environ.get("AB_REPS", "3"))
t = synth_config(cfg).typed(dpathsim.METAPATHS[CONFIGS[cfg][3]])
ref = None
for name, vs, sym in (("plain+vs", True, False), ("plain", False, False), ("sym", False, True)):
    if vs and W != 16384:
        continue
    if os.environ.get("AB_ONLY") and name != os.environ["AB_ONLY"]:
        continue
    eng = build_engine(t, tile_w=W, venue_skip=vs)
    eng.sym = sym
    eng.band = int(os.environ.get("AB_BAND", "1"))
    eng.sym_band = eng.band
    eng.sym_rec_per_row = int(os.environ.get("AB_REC", "160"))
    eng.topk(K); torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(); o = eng.topk(K); e1.record(); torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    o = [a.cpu().numpy() for a in o]
    dig = hashlib.sha1(b"".join(a.tobytes() for a in o)).hexdigest()[:16]
    extra = f" records {eng.check_sym()}" if sym else ""
    w = eng.tensor("topk_ws")[:256].view(torch.int64).cpu().tolist()
    if w[15]:
        extra += f" candidates {w[15]} inserted {w[16]} (rest pass)"
        st = max(w[12], 1)
        extra += (f"\n  rest-pass cycles per wave-stage: scatter {w[8] / st:.0f} flush+thr {w[9] / st:.0f} "
                  f"prefetch {w[10] / st:.0f} epilogue {w[11] / st:.0f} (stages {w[12]})")
    print(f"{cfg} W={W} k={K} {name}: {best:.2f} ms digest {dig} counts {eng.kernel_counts()}{extra}",
          flush=True)
    if ref is None:
        ref = o
    else:
        bad = np.flatnonzero((o[0] != ref[0]).any(1) | (o[1] != ref[1]).any(1) |
                             (o[2].view(np.int64) != ref[2].view(np.int64)).any(1))
        print(f"  vs first: {len(bad)} rows differ {bad[:5].tolist()}", flush=True)
    del eng
    torch.cuda.empty_cache()
