"""Predict the N-GPU step with the N > 1 build's tile split, on ONE GPU.

For world = 2, 4, 8: every rank's slices are built and recorded first (the
engine's split path with a recording stand-in for the all-gather); then each
rank's whole build is timed (events, eng.build) with an all-gather that copies
the recorded slices into place (a device copy of the gathered bytes: the
receive side's HBM writes; the xGMI transfer itself is modelled below), and the
hot kernel over each rank's row shard (bench.py's plan); and (round 5) the
replicated build and the shard's top-k enqueued back to back in one event
span, as bench.py's step runs them, plus the result gather to rank 0 over one
xGMI link per peer ("joint_replicated_speedup" against the same span at
N = 1).  Predicted step =
max over ranks of (build + shard kernel) + the modelled all-gather
(gathered bytes * (N-1)/N / XGMI_GBPS, default 150 GB/s = one xGMI link's worth:
every rank sends its slice to N-1 peers).  Prints JSON lines."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "distributed-pathsim_amd"))
import numpy as np
import torch

from dpathsim.dist import balanced_bounds
from dpathsim.engine import PathSimEngine, build_engine
from dpathsim.synth import CONFIGS, synth_config
import dpathsim

cfg = os.environ.get("SB_CONFIG", "config3")
k = int(os.environ.get("SB_K", str(CONFIGS[cfg][4])))
XGMI = float(os.environ.get("XGMI_GBPS", "150"))
t = synth_config(cfg).typed(dpathsim.METAPATHS[CONFIGS[cfg][3]])
NA = t.n_authors


class Split:
    def __init__(self, rank, world, slices=None, maxima=None):
        self.rank, self.world, self.slices = rank, world, slices
        self.caps = {}                  # the engine's plan, keyed by graph and width
        self.sent, self.calls, self.bytes = [], 0, 0
        self.seen, self.maxima = [], maxima

    def allgather(self, send, recv):
        if self.slices is None:
            self.sent.append(send.clone())
            recv.zero_()
        else:
            src = self.slices[self.calls]
            recv.copy_(src)
            self.bytes += src.numel() * src.element_size()
        self.calls += 1

    def allreduce_max(self, v):      # the plan: every rank's real slice size
        self.seen.append(int(v))
        return int(self.maxima[len(self.seen) - 1]) if self.maxima else int(v)


def ev_time(fn, reps=3):
    best = 1e30
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best


ref = build_engine(t)
ref.topk(k, 0, 20000)
full = ev_time(lambda: ref.topk(k), 2)
build1 = ev_time(lambda: ref.build(check=False))
# the step as bench.py runs it: build and top-k enqueued back to back, one
# event span (the host's enqueue of the top-k overlaps the build's GPU time)
joint1 = ev_time(lambda: (ref.build(check=False), ref.topk(k)), 2)
print(json.dumps({"config": cfg, "world": 1, "hot_ms": full, "build_ms": build1,
                  "joint_step_ms": joint1}), flush=True)
# result gather to rank 0 (bench's packed 8-byte words): each peer's rows over
# its own xGMI link to rank 0
RES_B = 8 * k
for world in (2, 4, 8):
    # record every rank's slices with the exact plan capacities
    sent = []
    for r in range(world):
        e = PathSimEngine(t)
        e.split = Split(r, world)
        e.upload().build(check=False)
        torch.cuda.synchronize()
        sent.append((e.split.sent, e.split.seen))
        del e
    maxima = [max(s[1][i] for s in sent) for i in range(len(sent[0][1]))]
    sent = []
    for r in range(world):
        e = PathSimEngine(t)
        e.split = Split(r, world, maxima=maxima)
        e.upload().build(check=False)
        torch.cuda.synchronize()
        sent.append(e.split.sent)
        del e
    gathered = [torch.cat([s[i] for s in sent]) for i in range(len(sent[0]))]
    gbytes = sum(g.numel() * g.element_size() for g in gathered)
    ag_ms = gbytes * (world - 1) / world / (XGMI * 1e9) * 1e3
    bounds = balanced_bounds(ref.row_work(), world)
    rows = []
    for r in range(world):
        e = PathSimEngine(t)
        e.split = Split(r, world, slices=gathered, maxima=maxima)
        e.upload()

        def step(e=e):
            e.split.calls = 0
            e.build(check=False)
        b_ms = ev_time(step)
        a, b = bounds[r]
        s_ms = ev_time(lambda a=a, b=b: ref.topk(k, a, b), 2)
        j_ms = ev_time(lambda a=a, b=b: (ref.build(check=False), ref.topk(k, a, b)), 2)
        rows.append((b_ms, s_ms, j_ms, b - a))
        del e
        torch.cuda.empty_cache()
    step_ms = max(b + s for b, s, _, _ in rows) + ag_ms
    repl_ms = max(s for _, s, _, _ in rows) + build1
    res_ms = max(n for _, _, _, n in rows) * RES_B / (XGMI * 1e9) * 1e3
    joint_ms = max(j for _, _, j, _ in rows) + res_ms
    print(json.dumps({"config": cfg, "world": world,
                      "build_ms": [round(b, 3) for b, _, _, _ in rows],
                      "shard_ms": [round(s, 2) for _, s, _, _ in rows],
                      "joint_replicated_step_ms": [round(j, 2) for _, _, j, _ in rows],
                      "result_gather_model_ms": res_ms,
                      "joint_replicated_speedup": joint1 / joint_ms,
                      "gathered_MB": gbytes / 1e6, "allgather_model_ms": ag_ms,
                      "predicted_step_ms": step_ms,
                      "predicted_speedup": (full + build1) / step_ms,
                      "replicated_build_step_ms": repl_ms,
                      "replicated_build_speedup": (full + build1) / repl_ms}), flush=True)
