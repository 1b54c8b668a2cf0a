"""Tail of the hot kernel: time the heaviest rows alone (one row = one wave)
and in groups, against their row_work estimate."""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-pathsim_amd"))
import numpy as np
import torch
from dpathsim.engine import build_engine
from dpathsim.synth import synth_config
t = synth_config(os.environ.get("HR_CONFIG", "config3")).typed()
eng = build_engine(t)
w = eng.row_work().cpu().numpy()
d = np.diff(eng.tensor("c_ptr")[: t.n_authors + 1].cpu().numpy())
order = np.argsort(-w, kind="stable")
def timed(rows, reps=2):
    best = 1e30
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); eng.topk_rows(10, rows); e1.record(); torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best
eng.topk_rows(10, order[:100])
for i in list(range(8)) + [15, 31, 63, 127, 255, 1023, 4095]:
    x = int(order[i])
    print(json.dumps({"rank": i, "row": x, "work": int(w[x]), "venues": int(d[x]),
                      "ms_alone": round(timed(np.array([x])), 3)}), flush=True)
for n in (16, 256, 4096, 65536):
    print(json.dumps({"heaviest_n": n, "ms": round(timed(order[:n]), 3),
                      "work_share": float(w[order[:n]].sum() / w.sum())}), flush=True)
