"""Round 6: the hot launch's ramp-down (profiling build, DPATHSIM_ABLATE=16):
every wave's realtime start / end stamps and the start of its last row, on the
full config3 launch (the bench's: heavy rows split).  Prints the distribution
of wave end times, the idle wave-time share at the end of the launch, and the
slowest last rows (dequeue position r: 0.. the split pieces, then rows
heaviest first)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-pathsim_amd"))
import numpy as np
import torch

from dpathsim.engine import build_engine
from dpathsim.synth import synth_config

cfg = os.environ.get("AB_CONFIG", "config3")
eng = build_engine(synth_config(cfg).typed())
R = eng.typed.n_authors
os.environ["DPATHSIM_ABLATE"] = "16"
for rows in ((0, R), (0, R // 8), (R // 2, R // 2 + R // 8)):
    eng.topk(10, 0, 20000)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    eng.topk(10, *rows)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    w = eng.tensor("topk_ws").view(torch.int64)[64: 64 + 4 * 16384].view(-1, 4).cpu().numpy()
    w = w[w[:, 1] > 0]
    t0 = w[:, 0].min()
    st, en, ls = (w[:, 0] - t0) / 1e5, (w[:, 1] - t0) / 1e5, (w[:, 2] - t0) / 1e5   # ms (100 MHz)
    T = en.max()
    busy = (en - st).sum() / (len(w) * T)
    last = en - ls
    q = np.percentile(en, [0, 10, 50, 90, 99, 100])
    print(f"{cfg} rows {rows}: launch {ms:.2f} ms (events), {len(w)} waves, span {T:.2f} ms; "
          f"wave end percentiles 0/10/50/90/99/100: " + " ".join(f"{v:.2f}" for v in q) +
          f"; busy share {busy:.3f}; start spread {st.max():.3f} ms", flush=True)
    late = st > 0.01 * T
    print(f"  start percentiles 50/80/85/90/95/99: " + " ".join(f"{v:.3f}" for v in np.percentile(st, [50, 80, 85, 90, 95, 99]))
          + f"; waves starting after 1% of the span: {int(late.sum())} ({late.mean():.3f}); "
          f"their mean start {st[late].mean() if late.any() else 0:.2f} ms", flush=True)
    bid = np.flatnonzero(w[:, 1] > 0)
    print(f"  late waves by block index (first 20): {np.flatnonzero(late)[:20].tolist()}", flush=True)
    order = np.argsort(-en)[:8]
    print("  latest waves: " + "; ".join(f"end {en[i]:.2f} last row r={int(w[i, 3])} took {last[i]:.2f}"
                                          for i in order), flush=True)
    print(f"  last-row duration percentiles 50/90/99/max: " +
          " ".join(f"{v:.3f}" for v in np.percentile(last, [50, 90, 99, 100])), flush=True)
