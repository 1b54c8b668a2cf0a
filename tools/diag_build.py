"""Build phases of one config (DIAG_CONFIG, default config4/APTPA) with timing,
printing as it goes (diagnostics for slow builds)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-pathsim_amd"))
import torch
from dpathsim.engine import PathSimEngine
from dpathsim.graph import METAPATHS
from dpathsim.synth import CONFIGS, synth_config
cfg = os.environ.get("DIAG_CONFIG", "config4")
t0 = time.perf_counter()
t = synth_config(cfg).typed(METAPATHS[CONFIGS[cfg][3]])
print(f"synth {time.perf_counter() - t0:.1f} s", flush=True)
eng = PathSimEngine(t).upload()
print(f"upload+bounds {time.perf_counter() - t0:.1f} s {eng.bounds}", flush=True)
for i in range(3):
    eng.build(timed=True)
    print({k: round(v, 3) for k, v in eng.info.phase_ms.items()}, flush=True)
t1 = time.perf_counter(); w = eng.row_work(); torch.cuda.synchronize()
print(f"row_work {1e3 * (time.perf_counter() - t1):.2f} ms", flush=True)
t1 = time.perf_counter(); eng.topk(10, 0, 20000); torch.cuda.synchronize()
print(f"topk 20k rows {1e3 * (time.perf_counter() - t1):.2f} ms", flush=True)
