"""Hot-kernel A/B across tile widths and waves per row on a config (all rows by
default): times eng.topk for each (W, NW) and checks the outputs are
bit-identical to the first run's."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-pathsim_amd"))
import numpy as np
import torch
from dpathsim.synth import synth_config, CONFIGS
from dpathsim.engine import build_engine

cfg = os.environ.get("AB_CONFIG", "config3")
K = int(os.environ.get("AB_K", str(CONFIGS[cfg][4])))
# cases "W:NW" (tile width : waves per workgroup, DPATHSIM_NW)
cases = [tuple(int(v) for v in c.split(":")) for c in os.environ.get("AB_CASES", "32768:4,8192:1").split(",")]
import dpathsim
from dpathsim import _lib
for kv in filter(None, os.environ.get("AB_TUNE", "").split(",")):   # "key=value,..."
    key, val = (int(v) for v in kv.split("="))
    _lib.call("dps_set_tuning", key, val)
t = synth_config(cfg).typed(dpathsim.METAPATHS[CONFIGS[cfg][3]])
R = int(os.environ.get("AB_ROWS", str(t.n_authors)))
ref = None
eng, W0 = None, None
for W, NW in cases:
    if W != W0:
        eng = None
        torch.cuda.empty_cache()
        from dpathsim.engine import PathSimEngine
        eng = PathSimEngine(t, tile_w=W)
        if os.environ.get("AB_NHEAVY"):
            eng.n_heavy = int(os.environ["AB_NHEAVY"])
        # optimistic 4-bit passes (engine.opt_passes, dps_cct_ext.tile_sum): on in
        # A/B runs only with AB_OPT=1 (the engine default is off)
        eng.opt_passes = os.environ.get("AB_OPT", "0") == "1"
        eng.dual_build = os.environ.get("AB_DUAL", "1") == "1"   # one-walk tile build (round 6)
        if os.environ.get("AB_SPLIT"):      # "rows:pieces" of the heavy-row split
            eng.split_rows, eng.pieces = (int(v) for v in os.environ["AB_SPLIT"].split(":"))
        eng.upload().build()
        W0 = W
        eng.build(timed=True)
        ph = eng.info.phase_ms
        print("  build ms: " + " ".join(f"{k} {v:.3f}" for k, v in ph.items() if k != "host_total")
              + f" total {sum(v for k, v in ph.items() if k != 'host_total'):.3f}", flush=True)
    os.environ["DPATHSIM_NW"] = str(NW)
    eng.topk(K, 0, min(R, 20000)); torch.cuda.synchronize()
    if True:
        best = 1e30
        for _ in range(int(os.environ.get("AB_REPS", "2"))):
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record(); o = eng.topk(K, 0, R); e1.record(); torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1))
        o = [a.cpu().numpy() for a in o]
        import hashlib
        dig = hashlib.sha1(b"".join(a.tobytes() for a in o)).hexdigest()[:16]
        kc = eng.kernel_counts()
        print(f"{cfg} W={W} NW={NW}: {best:.2f} ms for {R} rows (k={K}) digest {dig} "
              f"passes {kc['passes']} chunks {kc['chunks']} redo {kc.get('opt_redo', 0)}", flush=True)
        if ref is None:
            ref = o
        else:
            bad = np.flatnonzero((o[0] != ref[0]).any(1) | (o[1] != ref[1]).any(1) |
                                 (o[2].view(np.int64) != ref[2].view(np.int64)).any(1))
            print(f"  vs first: {len(bad)} rows differ {bad[:5].tolist()}", flush=True)
