"""Streaming GEXF loader at scale: write a synthetic config (default config3,
1M authors / 3M papers / 5k venues, ~10.5M edges) with write_gexf, read it
back with the streaming read_gexf, check the round trip, report MB/s and the
peak RSS.  CPU only."""
import json, os, resource, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-pathsim_amd"))
import numpy as np
from dpathsim.gexf import read_gexf, write_gexf
from dpathsim.synth import synth_config
cfg = os.environ.get("LS_CONFIG", "config3")
path = os.environ.get("LS_PATH", f"/tmp/{cfg}.gexf")
g = synth_config(cfg)
t0 = time.perf_counter(); write_gexf(g, path); tw = time.perf_counter() - t0
mb = os.path.getsize(path) / 1e6
t0 = time.perf_counter(); h = read_gexf(path); tr = time.perf_counter() - t0
# the reader returns edges in networkx adjacency order (by source node), so
# compare the edge multisets
key = lambda gr: np.sort(gr.edge_src.astype(np.int64) * gr.n_nodes + gr.edge_dst)
ok = (h.n_nodes == g.n_nodes and h.n_edges == g.n_edges
      and np.array_equal(h.node_type_idx, g.node_type_idx) and np.array_equal(key(h), key(g)))
print(json.dumps({"config": cfg, "bytes_mb": round(mb, 1), "nodes": h.n_nodes, "edges": h.n_edges,
                  "write_s": round(tw, 1), "write_mb_s": round(mb / tw, 1),
                  "read_s": round(tr, 1), "read_mb_s": round(mb / tr, 1),
                  "read_edges_per_s": round(h.n_edges / tr),
                  "peak_rss_gb": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6, 2),
                  "roundtrip_exact": bool(ok)}), flush=True)
os.remove(path)
