"""GPU: the reference-compatible surface (DPathSim_APVPA class, run() log) vs the oracle."""
import os
import re

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TIMING = re.compile(r"^\*\*\*(Stage|Overall) done in: [0-9.e+-]+$")


@pytest.fixture(scope="module")
def graph_and_engine(dblp_small_tuples):
    from dpathsim.engine import build_engine
    from dpathsim.graph import Graph
    g = Graph.from_tuples(*dblp_small_tuples)
    return g, build_engine(g.typed(), tile_w=256)


@pytest.mark.parametrize("source", ["author_7007701", "author_395340", "author_1238349"])
def test_run_log_matches_oracle(tmp_path, graph_and_engine, dblp_small_tuples, source):
    import pathsim_oracle as po
    from dpathsim.compat import DPathSim_APVPA
    g, eng = graph_and_engine
    out = tmp_path / "run.log"
    DPathSim_APVPA(g, eng, source, str(out)).run()
    lines = out.read_text(encoding="utf-8").splitlines()
    assert TIMING.match(lines[-1]) and lines[-1].startswith("***Overall")
    body = [ln for ln in lines if not TIMING.match(ln) and ln != "---"]
    expect = po.single_source_log_lines(po.OracleGraph(*dblp_small_tuples), source)
    assert body == expect
    # 5 lines per target (:42-64): pairwise, target gw, score, stage time, ---
    assert len(lines) == 1 + 5 * 769 + 1


def test_reference_default_source_absent_raises_keyerror(tmp_path, graph_and_engine):
    """'Jiawei Han' is not in dblp_small: global walk 0, then KeyError at :56."""
    from dpathsim.compat import DPathSim_APVPA, find_author_node_id_by_name
    g, eng = graph_and_engine
    src = find_author_node_id_by_name(g, "Jiawei Han")
    assert src is None
    d = DPathSim_APVPA(g, eng, src, str(tmp_path / "x.log"))
    assert d.metapath_global_walk(src) == 0
    with pytest.raises(KeyError):
        d.run()
    d.output_file.close()   # like the reference, nothing is flushed before the KeyError
    text = (tmp_path / "x.log").read_text()
    assert text.startswith("Source author global walk: 0\nPairwise authors walk author_395340: 0\n")


def test_methods_match_bruteforce_motif(graph_and_engine, dblp_small_tuples):
    import motif_bruteforce as mb
    from dpathsim.compat import DPathSim_APVPA
    g, eng = graph_and_engine
    v, e = dblp_small_tuples
    d = DPathSim_APVPA.__new__(DPathSim_APVPA)
    d.dblp_graph, d.dblp_graphframe = g, eng
    rng = np.random.default_rng(3)
    ids = [x[0] for x in v]
    for a in rng.choice(ids, 12, replace=False):
        assert d.metapath_global_walk(a) == mb.motif_count(v, e, a)
        b = ids[int(rng.integers(len(ids)))]
        assert d.metapath_pairwise_walk(a, b) == mb.motif_count(v, e, a, b)
