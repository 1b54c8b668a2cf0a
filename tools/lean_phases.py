"""Phase cycles of the lean hot kernel (profiling build, DPATHSIM_ABLATE=16):
shader-clock cycles per wave-stage in scatter / flush+thresholds / next-stage
prefetch / epilogue, on the full config3 launch."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-pathsim_amd"))
import torch
from dpathsim.synth import synth_config
from dpathsim.engine import build_engine

eng = build_engine(synth_config(os.environ.get("AB_CONFIG", "config3")).typed(), tile_w=int(os.environ.get("AB_W", "16384")))
R = eng.typed.n_authors
for ab in ("0", "16"):
    os.environ["DPATHSIM_ABLATE"] = ab
    eng.topk(10, 0, 20000); torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record(); eng.topk(10, 0, R); e1.record(); torch.cuda.synchronize()
    print(f"ablate {ab}: {e0.elapsed_time(e1):.2f} ms", flush=True)
c = eng.tensor("topk_ws")[:512].view(torch.int64).cpu().tolist()
st = max(c[12], 1)
names = ["scatter", "flush+thresholds", "prefetch", "epilogue"]
tot = sum(c[8:12])
print(f"  prefetch split: refilter+stage_make {c[13] / st:.0f}, issue batch 0 {c[14] / st:.0f}, rest {(c[10] - c[13] - c[14]) / st:.0f}", flush=True)
print(f"candidates scored {c[15]} ({c[15] / st:.1f} per stage, {c[15] / R:.1f} per row), "
      f"inserted {c[16]} ({c[16] / R:.1f} per row)", flush=True)
print(f"passes over u8 half tiles {c[17]} ({c[17] / st:.3f} of stages), with wider counters "
      f"{c[18]} ({c[18] / st:.4f})", flush=True)
print(f"stages {st} ({st / R:.1f} per row); cycles per wave-stage: " +
      " ".join(f"{n} {c[8 + i] / st:.0f} ({c[8 + i] / tot:.0%})" for i, n in enumerate(names)), flush=True)
nb = max(sum(c[19:23]), 1)
print(f"epilogue blocks {nb} ({nb / st:.2f} per stage): above counter width {c[19] / nb:.1%}, "
      f"prefilter empty {c[20] / nb:.1%}, exact empty {c[21] / nb:.1%}, with candidates {c[22] / nb:.1%}; "
      f"extraction rounds {c[23]} ({c[23] / max(c[22], 1):.2f} per candidate block)", flush=True)
edges = ["0", "1-16", "17-64", "65-128", "129-192", "193-384", "385-768", ">768"]
npass = max(sum(c[24:32]), 1)
epi = max(sum(c[40:48]), 1)
print("passes by the stage's chunk count (share of passes / of chunks / of epilogue cycles, "
      "epilogue cycles per pass):", flush=True)
for i, e in enumerate(edges):
    print(f"  {e:>8}: {c[24 + i] / npass:6.1%} {c[32 + i] / max(sum(c[32:40]), 1):6.1%} "
          f"{c[40 + i] / epi:6.1%}  {c[40 + i] / max(c[24 + i], 1):7.0f}", flush=True)
