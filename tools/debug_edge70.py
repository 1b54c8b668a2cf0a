"""Round 6: the debug build's mismatch in test_random_multigraphs_vs_oracle[70]
(general kernel, tile_w 256, k = 70): rebuild the test's graphs, and for the
first trial that differs print the graph size and the differing rows (slots,
counts, scores) of the library DPATHSIM_LIB points at and of the oracle."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-pathsim_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import numpy as np

import pathsim_oracle as po
from dpathsim.engine import build_engine
from dpathsim.graph import Graph

k = int(os.environ.get("DBG_K", "70"))
tile_w = int(os.environ.get("DBG_W", "256"))
rng = np.random.default_rng(k)
types = ["author", "paper", "venue", "topic"]
rels = ["author_of", "submit_at", "cites"]
bad = 0
for trial in range(25):
    n = int(rng.integers(3, 90))
    ty = rng.choice(types, size=n, p=[0.45, 0.35, 0.15, 0.05])
    v = [(f"n{i}", f"L{i}", str(ty[i])) for i in range(n)]
    m = int(rng.integers(0, 6 * n))
    e = [(f"n{int(a)}", f"n{int(b)}", str(r)) for a, b, r in
         zip(rng.integers(0, n, m), rng.integers(0, n, m), rng.choice(rels, size=m))]
    t = Graph.from_tuples(v, e).typed()
    if t.n_authors == 0:
        continue
    eng = build_engine(t, tile_w=tile_w)
    gi, gc, gs = (a.cpu().numpy() for a in eng.topk(k))
    oi, oc, os_ = po.allpairs_topk(po.OracleGraph(v, e), k)
    rows = np.flatnonzero((gi != oi).any(1) | (gc != oc).any(1) | (gs.view(np.int64) != os_.view(np.int64)).any(1))
    print(f"trial {trial}: n {n} authors {t.n_authors} edges {m} differing rows {len(rows)}", flush=True)
    for x in rows[:4]:
        pos = np.flatnonzero((gi[x] != oi[x]) | (gc[x] != oc[x]))
        print(f"  row {x}: first differing slots {pos[:8].tolist()}", flush=True)
        lo = max(0, int(pos[0]) - 2) if len(pos) else 0
        print(f"    got  idx {gi[x, lo:lo + 10].tolist()} cnt {gc[x, lo:lo + 10].tolist()} "
              f"score {gs[x, lo:lo + 10].tolist()}", flush=True)
        print(f"    want idx {oi[x, lo:lo + 10].tolist()} cnt {oc[x, lo:lo + 10].tolist()} "
              f"score {os_[x, lo:lo + 10].tolist()}", flush=True)
        filled = int((gc[x] > 0).sum())
        print(f"    got positive {filled}, want positive {int((oc[x] > 0).sum())}", flush=True)
    bad += len(rows) > 0
    if bad >= 3:
        break
print("done", flush=True)
