"""Round 6: what the hot launch's dequeue order costs at the end of a launch.

Phase "prof" (profiling build, DPATHSIM_LIB=.../libdpathsim_prof.so): one launch
over the rows of each range with DPATHSIM_ABLATE=16; the kernel records every
dequeue slot's wall time (100 MHz realtime ticks) and accumulator passes
(counter[64 + 4 * 16384 + r]).  Prints, per range: time and passes by dequeue
position, the last slots' times, rank correlations of a row's time with the
keys available before the launch, and a list-scheduling model of the launch
(ROW_WAVES waves take the next slot when free) for several orders.  Saves the
records to ROW_OUT (npz).

Phase "time" (in-tree library): the real launches of each range with the
dequeue key = row_terms (the default), the profiled time, the profiled passes
and the candidate predictors, event-timed ABAB.  Every order gives identical
lists (digest checked)."""
import heapq
import hashlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-pathsim_amd"))
import numpy as np
import torch

from dpathsim.engine import build_engine
from dpathsim.synth import synth_config

cfg = os.environ.get("AB_CONFIG", "config3")
phase = os.environ.get("ROW_PHASE", "prof")
out = os.environ.get("ROW_OUT", "gpurun_out/row_times.npz")
waves = int(os.environ.get("ROW_WAVES", "4608"))
reps = int(os.environ.get("ROW_REPS", "3"))
K = 10
eng = build_engine(synth_config(cfg).typed())
NA = eng.typed.n_authors
ranges = [(0, NA // 8), (NA // 2, NA // 2 + NA // 8), (0, NA)]
if os.environ.get("ROW_RANGES"):
    ranges = [tuple(int(v) for v in r.split(":")) for r in os.environ["ROW_RANGES"].split(",")]
d = eng._dev
terms = d["row_terms"][:NA].to(torch.int64)
cp = d["c_ptr"][: NA + 1].to(torch.int64)
deg = (cp[1:] - cp[:-1]).to(torch.int64)


def sched(dur, n):
    """makespan of greedy list scheduling of `dur` (in order) on n waves"""
    h = [0.0] * min(n, len(dur))
    heapq.heapify(h)
    for t in dur:
        heapq.heappush(h, heapq.heappop(h) + float(t))
    return max(h)


def spearman(a, b):
    ra = np.argsort(np.argsort(a)).astype(np.float64)
    rb = np.argsort(np.argsort(b)).astype(np.float64)
    return float(np.corrcoef(ra, rb)[0, 1])


if phase == "prof":
    os.environ["DPATHSIM_ABLATE"] = "16"
    ws = eng.tensor("topk_ws").view(torch.int64)
    base = 64 + 4 * 16384
    saved = {}
    for (b, e) in ranges:
        eng.topk(K, 0, 20000)
        torch.cuda.synchronize()
        ws[base: base + (1 << 21)].zero_()
        torch.cuda.synchronize()
        eng.topk(K, b, e)
        torch.cuda.synchronize()
        dq = eng._last_dq.cpu().numpy().astype(np.int64)
        n = len(dq)
        rec = ws[base: base + n].cpu().numpy().view(np.uint64)
        dur = (rec >> np.uint64(32)).astype(np.float64) / 100.0        # us
        npass = (rec & np.uint64(0xFFFFFFFF)).astype(np.int64)
        n_p = n - (e - b)                                                # extra piece slots
        M = n_p // 15 if n_p else 0                                      # 16 pieces per split row
        n_piece = M * 16
        rows = dq[n_piece:]
        saved[f"{b}_{e}_dq"] = dq
        saved[f"{b}_{e}_dur"] = dur
        saved[f"{b}_{e}_pass"] = npass
        print(f"{cfg} rows [{b}, {e}): {n} slots ({n_piece} pieces), total wave time {dur.sum()/1e3:.1f} ms, "
              f"{npass.sum()} passes, zero-time slots {(rec == 0).sum()}", flush=True)
        q = np.linspace(0, n, 21).astype(int)
        print("  by dequeue position (20 bins): mean us / mean passes")
        print("   " + " ".join(f"{dur[q[i]:q[i+1]].mean():.0f}/{npass[q[i]:q[i+1]].mean():.0f}" for i in range(20)))
        for f in (0.005, 0.01, 0.02, 0.05):
            m = max(1, int(f * n))
            t = dur[-m:]
            print(f"  last {f*100:.1f}% ({m} slots): time us p50/p90/p99/max "
                  + " ".join(f"{v:.0f}" for v in np.percentile(t, [50, 90, 99, 100]))
                  + f"; passes mean {npass[-m:].mean():.1f}")
        rd, rp = dur[n_piece:], npass[n_piece:]
        tr = terms[torch.from_numpy(rows).to(terms.device)].cpu().numpy()
        dg = deg[torch.from_numpy(rows).to(terms.device)].cpu().numpy()
        print(f"  rank corr of row time with: passes {spearman(rd, rp):.3f}, terms {spearman(rd, tr):.3f}, "
              f"venues {spearman(rd, dg):.3f}")
        pc = dur[:n_piece]
        for name, key in (("as launched", None), ("by time (LPT)", rd), ("by passes", rp),
                          ("by terms", tr)):
            o = np.arange(len(rd)) if key is None else np.argsort(-key, kind="stable")
            ms = sched(np.concatenate([pc, rd[o]]), waves) / 1e3
            print(f"  list model, {waves} waves, {name}: makespan {ms:.3f} ms (ideal {dur.sum()/waves/1e3:.3f})")
    np.savez(out, **saved)
    print("saved", out)
else:
    rec = np.load(out)
    for (b, e) in ranges:
        dq = rec[f"{b}_{e}_dq"]
        n_piece = len(dq) - (e - b)
        n_piece = n_piece // 15 * 16 if n_piece else 0
        rows = dq[n_piece:] - b
        keys = {"terms": None}
        for nm, arr in (("time", rec[f"{b}_{e}_dur"]), ("passes", rec[f"{b}_{e}_pass"].astype(np.float64))):
            w = np.zeros(e - b)
            w[rows] = arr[n_piece:]
            # the split rows keep their place at the front: their key above every other
            w[dq[:n_piece:16] - b] = w.max() * 4 + 1
            keys[nm] = torch.from_numpy(np.round(w * 16).astype(np.int64) + 1).to(eng.device)
        res = {nm: [] for nm in keys}
        dig = {}
        for _ in range(reps):
            for nm, kw in keys.items():
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                idx, cnt, sc = eng.topk(K, b, e, row_work=kw)
                e1.record()
                torch.cuda.synchronize()
                res[nm].append(e0.elapsed_time(e1))
                h = hashlib.sha1(idx.cpu().numpy().tobytes() + cnt.cpu().numpy().tobytes()).hexdigest()[:16]
                dig.setdefault(nm, h)
                assert dig[nm] == h
        print(f"{cfg} rows [{b}, {e}): " + "; ".join(
            f"{nm} {np.median(v):.3f} ms (min {min(v):.3f}) digest {dig[nm]}" for nm, v in res.items()), flush=True)
        assert len(set(dig.values())) == 1, "orders disagree"
