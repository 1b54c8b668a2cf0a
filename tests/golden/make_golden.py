"""Generate the committed golden fixtures under tests/golden/ (run once, here).

Reads two DATA files of the reference (never its sources):
  * /root/reference/dblp/dblp_small.gexf            -- the small DBLP graph
  * /root/reference/output/d_pathsim_output_20180417_020445.log -- the 2018 run log

and writes:
  * dblp_small_graph.json.gz  -- the graph exactly as the reference loader hands it
    to Spark (``DPathSim_APVPA.py:114-129``: vertices (id,label,node_type) in node
    order, edges (src,dst,relationship) in networkx edge order), so tests on the
    GPU box (no /root/reference there) see the same input.
  * log_triples.json          -- 81 (target, pairwise walk, target global walk,
    score repr) stages of the log + the source global walk (log:1).
  * small_globalwalk_golden.json -- the logged target global walks that the
    dblp_small restatement reproduces (row-sum semantics).
  * dblp_small_expected.npz   -- oracle C (CSR), s, g, top-10 for all 770 authors,
    whole-graph invariants.  Produced by oracle/pathsim_oracle.py, which is itself
    checked here against the log vectors and the brute-force motif counter.

Usage:  python tests/golden/make_golden.py
"""
import gzip
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import motif_bruteforce  # noqa: E402
import pathsim_oracle as po  # noqa: E402

REF = "/root/reference"
GEXF = os.path.join(REF, "dblp", "dblp_small.gexf")
LOG = os.path.join(REF, "output", "d_pathsim_output_20180417_020445.log")


def parse_log(path):
    lines = open(path, encoding="utf-8").read().split("\n")
    m = re.match(r"Source author global walk: (\d+)$", lines[0])
    gx = int(m.group(1))
    stages = []
    i = 1
    while i + 4 < len(lines):
        a = re.match(r"Pairwise authors walk (\S+): (\d+)$", lines[i])
        b = re.match(r"Target author global walk: (\d+)$", lines[i + 1])
        c = re.match(r"Sim score (.*) - (.*): (\S+)$", lines[i + 2])
        d = re.match(r"\*\*\*Stage done in: (\S+)$", lines[i + 3])
        if not (a and b and c and d and lines[i + 4] == "---"):
            break
        stages.append({
            "line": i + 1,                      # 1-based line of "Pairwise authors walk"
            "target_id": a.group(1), "pw": int(a.group(2)),
            "gy": int(b.group(1)), "gy_line": i + 2,
            "source_label": c.group(1), "target_label": c.group(2),
            "score_repr": c.group(3), "stage_seconds": float(d.group(1)),
        })
        i += 5
    return gx, stages


def main():
    gx, stages = parse_log(LOG)
    assert gx == 8423 and len(stages) == 81, (gx, len(stages))
    for s in stages:   # the score formula of :51-52 reproduces every logged score bit-exactly
        assert repr(2 * s["pw"] / (gx + s["gy"])) == s["score_repr"], s
    with open(os.path.join(HERE, "log_triples.json"), "w") as f:
        json.dump({"source_global_walk": gx, "source_label": stages[0]["source_label"],
                   "log": os.path.relpath(LOG, REF), "stages": stages}, f, indent=1)

    vertices, edges = po.load_gexf_networkx(GEXF)
    with gzip.open(os.path.join(HERE, "dblp_small_graph.json.gz"), "wt", encoding="utf-8") as f:
        json.dump({"source": "dblp/dblp_small.gexf via networkx.read_gexf "
                             "(DPathSim_APVPA.py:114-129 loader semantics)",
                   "vertices": vertices, "edges": edges}, f)

    g = po.OracleGraph(vertices, edges)
    # brute-force motif agreement on a sample of sources (and all pairs among them)
    sample = g.authors[:40] + g.authors[-10:]
    for a in sample:
        assert g.global_walk(a) == motif_bruteforce.motif_count(vertices, edges, a)
    for a in sample[:12]:
        for b in sample[:12]:
            assert g.pairwise_walk(a, b) == motif_bruteforce.motif_count(vertices, edges, a, b)

    small = []
    for s in stages:
        if s["target_id"] in g.author_ord and g.global_walk(s["target_id"]) == s["gy"]:
            small.append({"target_id": s["target_id"], "g": s["gy"], "log_line": s["gy_line"]})
    with open(os.path.join(HERE, "small_globalwalk_golden.json"), "w") as f:
        json.dump(small, f, indent=1)

    idx, cnt, sc = po.allpairs_topk(g, 10)
    M = (g.C @ g.C.T).toarray()
    inv = dict(sum_g=int(g.g.sum()), trace_M=int(np.trace(M)), sum_C=int(g.C.sum()),
               nnz_C=int(g.C.nnz), max_C=int(g.C.max()), nnz_M=int((M > 0).sum()),
               max_M=int(M.max()), max_offdiag_M=int((M - np.diag(np.diag(M))).max()),
               min_g=int(g.g.min()), max_g=int(g.g.max()),
               n_nodes=len(vertices), n_edges=len(edges), n_authors=len(g.authors),
               n_papers=len(g.papers), n_venues=len(g.mids))
    np.savez_compressed(
        os.path.join(HERE, "dblp_small_expected.npz"),
        c_ptr=g.C.indptr.astype(np.int64), c_col=g.C.indices.astype(np.int32),
        c_val=g.C.data.astype(np.int32), s=g.s, g=g.g,
        top10_idx=idx, top10_cnt=cnt, top10_score=sc,
        invariants=np.array(json.dumps(inv)))
    print(json.dumps(inv))
    print("log stages", len(stages), "small-graph global walks", len(small),
          [x["log_line"] for x in small])


if __name__ == "__main__":
    main()
