"""Round 6: the per-shard launch overhead, kernel by kernel.  Runs bench.py's
N-rank row shards of config3 (dps_shard_edges over the build's row work) one
after another on one GPU, each SHARD_REPS times, event-timed; run it under
`rocprofv3 --kernel-trace --stats` and summarise the trace with
`tools/shard_trace.py --summary <kernel_trace.csv>` (k_cct1, the dequeue list
and the piece merge per launch)."""
import csv
import os
import sys

if len(sys.argv) > 2 and sys.argv[1] == "--summary":
    rows = list(csv.DictReader(open(sys.argv[2])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # group the dispatches between consecutive k_cct1 launches' preceding k_work_key
    launches, cur = [], None
    for r in rows:
        n = r["Kernel_Name"]
        dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        if "k_work_key" in n:
            cur = {"start": int(r["Start_Timestamp"]), "kernels": []}
            launches.append(cur)
        if cur is not None:
            cur["kernels"].append((n.split("(")[0][:40], dt))
            cur["end"] = int(r["End_Timestamp"])
    for i, L in enumerate(launches):
        tot = (L["end"] - L["start"]) / 1e6
        ks = "; ".join(f"{n} {dt:.3f}" for n, dt in L["kernels"])
        print(f"launch {i}: span {tot:.3f} ms: {ks}")
    sys.exit(0)

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-pathsim_amd"))
import torch

from dpathsim.dist import shard_edges
from dpathsim.engine import build_engine
from dpathsim.synth import synth_config

world = int(os.environ.get("SHARD_WORLD", "8"))
reps = int(os.environ.get("SHARD_REPS", "2"))
eng = build_engine(synth_config(os.environ.get("AB_CONFIG", "config3")).typed())
NA = eng.typed.n_authors
e = shard_edges(eng.tensor("row_terms")[:NA], world).cpu().tolist()
eng.topk(10, 0, 20000)
torch.cuda.synchronize()
tot = []
for s in range(world):
    best = 1e30
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        eng.topk(10, e[s], e[s + 1])
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    tot.append(best)
    print(f"shard {s} rows [{e[s]}, {e[s + 1]}): {best:.3f} ms", flush=True)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
eng.topk(10, 0, NA)
e1.record()
torch.cuda.synchronize()
print(f"world {world}: shards sum {sum(tot):.3f} ms, max {max(tot):.3f}; one launch {e0.elapsed_time(e1):.3f} ms",
      flush=True)
