"""Round 6: the debug build's mismatch in test_split_rows_identical_lean[100-8192]
(u8 tiles, k = 100: the two-register top-k).  Runs the test's graph with and
without the heavy-row split, compares both with the C oracle, and describes
the rows that differ: split rows (pieces + merge) or whole rows, which side
matches the oracle, and the first difference."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-pathsim_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import numpy as np

import pathsim_oracle as po
from dpathsim.engine import build_engine
from dpathsim.synth import synth_dblp

K = int(os.environ.get("DBG_K", "100"))
W = int(os.environ.get("DBG_W", "8192"))
t = synth_dblp(40_000, 120_000, 400, seed=17).typed()
eng = build_engine(t, tile_w=W)
NA = t.n_authors
want = po.COracle.from_typed(t).topk(K, 0, NA)


def bad_rows(got, ref):
    gi, gc, gs = got
    oi, oc, os_ = ref
    return np.flatnonzero((gi != oi).any(1) | (gc != oc).any(1) |
                          (gs.view(np.int64) != os_.view(np.int64)).any(1))


whole = [a.cpu().numpy() for a in eng.topk(K, split_rows=0)]
print(f"lib {os.environ.get('DPATHSIM_LIB', 'release')}: W={W} k={K}", flush=True)
print(f"  whole vs oracle: {len(bad_rows(whole, want))} rows differ", flush=True)
for M, P in (((256, 16), (100, 3)) if os.environ.get("DBG_SPLIT", "1") == "1" else ()):
    got = [a.cpu().numpy() for a in eng.topk(K, 0, NA, split_rows=M, pieces=P)]
    dq = getattr(eng, "_last_dq", None)
    split = set(dq.cpu().numpy()[: M * P: P].tolist()) if dq is not None else set()
    b = bad_rows(got, want)
    ns = sum(1 for r in b if r in split)
    print(f"  split M={M} P={P} vs oracle: {len(b)} rows differ ({ns} of them split rows)", flush=True)
    for r in b[:3]:
        gi, gc, gs = (a[r] for a in got)
        oi, oc, os_ = (a[r] for a in want)
        d = np.flatnonzero((gi != oi) | (gc != oc))
        print(f"    row {r} ({'split' if r in split else 'whole'}): first slots differing {d[:8].tolist()}; "
              f"got idx {gi[d[:4]].tolist()} cnt {gc[d[:4]].tolist()}; want idx {oi[d[:4]].tolist()} "
              f"cnt {oc[d[:4]].tolist()}; got filled {int((gi >= 0).sum())} want {int((oi >= 0).sum())}",
              flush=True)
