import gzip, json, os, sys
import numpy as np
sys.path.insert(0, "distributed-pathsim_amd")
import torch
from dpathsim.graph import Graph
from dpathsim.engine import build_engine
d = json.load(gzip.open("tests/golden/dblp_small_graph.json.gz", "rt"))
v = [tuple(x) for x in d["vertices"]]; e = [tuple(x) for x in d["edges"]]
ex = np.load("tests/golden/dblp_small_expected.npz")
t = Graph.from_tuples(v, e).typed()
for W in (256, 512, 4096):
    for skip in (True, False):
        eng = build_engine(t, tile_w=W)
        eng.tile_skip = skip
        idx, cnt, sc = (a.cpu().numpy() for a in eng.topk(10))
        bad = np.flatnonzero((idx != ex["top10_idx"]).any(1) | (sc.view(np.int64) != ex["top10_score"].view(np.int64)).any(1))
        print(f"W={W} skip={skip}: {len(bad)} bad rows", bad[:10].tolist())
        for r in bad[:2]:
            print("  row", r, "got", idx[r].tolist(), cnt[r].tolist(), sc[r].tolist())
            print("  row", r, "exp", ex["top10_idx"][r].tolist(), ex["top10_cnt"][r].tolist(), ex["top10_score"][r].tolist())
