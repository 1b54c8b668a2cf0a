"""CPU: the oracle against the reference's golden vectors and the brute-force motif join."""
import os

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings, strategies as st

import motif_bruteforce as mb
import pathsim_oracle as po

REF_GEXF = "/root/reference/dblp/dblp_small.gexf"


def test_log_scores_reproduce_bit_exactly(log_triples):
    """81 logged (pw, gy, score) stages: score == 2*pw/(gx+gy) as IEEE fp64 (log:2-406)."""
    gx = log_triples["source_global_walk"]
    assert gx == 8423
    assert len(log_triples["stages"]) == 81
    for s in log_triples["stages"]:
        assert repr(2 * s["pw"] / (gx + s["gy"])) == s["score_repr"]
        num = np.float64(2 * s["pw"])
        den = np.float64(gx + s["gy"])
        assert repr(float(num / den)) == s["score_repr"]
        assert repr(float(po.scores_fp64([s["pw"]], [gx], [s["gy"]])[0])) == s["score_repr"]


def test_log_target_order_is_dblp_small_author_prefix(log_triples, dblp_small_tuples):
    v, _ = dblp_small_tuples
    authors = [x[0] for x in v if x[2] == "author"]
    assert [s["target_id"] for s in log_triples["stages"]] == authors[:81]


def test_small_graph_global_walks_match_log(dblp_small_tuples):
    """26 logged target global walks equal the dblp_small ROW SUM."""
    import json
    here = os.path.join(os.path.dirname(__file__), "golden", "small_globalwalk_golden.json")
    gold = json.load(open(here))
    assert len(gold) == 26
    g = po.OracleGraph(*dblp_small_tuples)
    for item in gold:
        assert g.global_walk(item["target_id"]) == item["g"]
    # the diagonal (textbook PathSim) would NOT reproduce them
    C = g.C
    diag_mismatch = 0
    for item in gold:
        r = g.author_ord[item["target_id"]]
        d = int(C[r].multiply(C[r]).sum())
        diag_mismatch += d != item["g"]
    assert diag_mismatch > 20


def test_dblp_small_invariants(dblp_small_tuples, dblp_small_expected):
    g = po.OracleGraph(*dblp_small_tuples)
    inv = dblp_small_expected["invariants"]
    M = (g.C @ g.C.T).toarray()
    assert int(g.g.sum()) == inv["sum_g"] == 79873
    assert int(np.trace(M)) == inv["trace_M"] == 2241
    assert int(g.C.sum()) == inv["sum_C"] == 1265
    assert g.C.nnz == inv["nnz_C"] == 971
    assert int((M > 0).sum()) == inv["nnz_M"] == 36150
    assert int(g.g.min()) == 1 and int(g.g.max()) == 1396
    assert np.array_equal(g.g, dblp_small_expected["g"])


def test_oracle_vs_bruteforce_dblp_small(dblp_small_tuples):
    v, e = dblp_small_tuples
    g = po.OracleGraph(v, e)
    rng = np.random.default_rng(0)
    for a in rng.choice(g.authors, 15, replace=False):
        assert g.global_walk(a) == mb.motif_count(v, e, a)
        b = g.authors[int(rng.integers(len(g.authors)))]
        assert g.pairwise_walk(a, b) == mb.motif_count(v, e, a, b)


def test_c_oracle_matches_python_oracle(dblp_small_tuples, dblp_small_expected):
    from dpathsim.graph import Graph
    t = Graph.from_tuples(*dblp_small_tuples).typed()
    co = po.COracle.from_typed(t)
    cp, cc, cv, s, g = co.export()
    ex = dblp_small_expected
    for a, b in ((cp, ex["c_ptr"]), (cc, ex["c_col"]), (cv, ex["c_val"]), (s, ex["s"]),
                 (g, ex["g"])):
        assert np.array_equal(a, b)
    idx, cnt, sc = co.topk(10, threads=2)
    assert np.array_equal(idx, ex["top10_idx"])
    assert np.array_equal(cnt, ex["top10_cnt"])
    assert np.array_equal(sc.view(np.int64), ex["top10_score"].view(np.int64))


# ---- hypothesis: small multigraphs with the reference's corner cases ----------
NODE_TYPES = ["author", "paper", "venue", "topic"]
RELS = ["author_of", "submit_at", "cites"]


@st.composite
def small_graphs(draw):
    n = draw(st.integers(2, 14))
    types = draw(st.lists(st.sampled_from(NODE_TYPES), min_size=n, max_size=n))
    vertices = [(f"n{i}", f"L{i}", types[i]) for i in range(n)]
    m = draw(st.integers(0, 40))
    edges = []
    for _ in range(m):
        s = draw(st.integers(0, n - 1))
        t = draw(st.integers(0, n - 1))
        r = draw(st.sampled_from(RELS))
        edges.append((f"n{s}", f"n{t}", r))
    return vertices, edges


@settings(max_examples=150, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(small_graphs())
def test_oracle_matches_motif_join(graph):
    """Parallel edges, untyped author_of sources, papers with 0/2+ venues, self loops."""
    v, e = graph
    g = po.OracleGraph(v, e)
    for a in [x[0] for x in v]:
        assert g.global_walk(a) == mb.motif_count(v, e, a)
        for b in [x[0] for x in v][:5]:
            assert g.pairwise_walk(a, b) == mb.motif_count(v, e, a, b)


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(small_graphs(), st.integers(1, 6))
def test_c_oracle_topk_matches_python_oracle(graph, k):
    from dpathsim.graph import Graph
    v, e = graph
    g = po.OracleGraph(v, e)
    t = Graph.from_tuples(v, e).typed()
    if t.n_authors == 0:
        return
    co = po.COracle.from_typed(t)
    a = po.allpairs_topk(g, k)
    b = co.topk(k, threads=1)
    for x, y in zip(a, b):
        assert np.array_equal(np.asarray(x).view(np.int64) if x.dtype == np.float64 else x,
                              np.asarray(y).view(np.int64) if y.dtype == np.float64 else y)


@pytest.mark.skipif(not os.path.exists(REF_GEXF), reason="reference data not present")
def test_networkx_loader_matches_fixture(dblp_small_tuples):
    v, e = po.load_gexf_networkx(REF_GEXF)
    assert (v, e) == dblp_small_tuples


# ---- the C oracle's shortcuts against the plain numpy restatement -------------
# Every full-size GPU parity test compares with the C oracle (COracle), which
# takes two shortcuts (oracle/pathsim_oracle.c): int32 accumulators when
# sum_v C[x,v] * max_y C[y,v] < 2^31 for every row, and no division when
# 2m < kth * den * (1 - 2^-40).  Here both are checked, on and forced off,
# against allpairs_topk (dense M rows + lexsort, no shortcut) on a 10k-author
# config3-shaped graph at k = 10 and 100, and on a graph whose path counts need
# int64 (the wide path taken by the proof, not by a switch).
def _typed_and_oracles(graph, k):
    from dpathsim.graph import APVPA
    t = graph.typed(APVPA)
    og = po.OracleGraph(graph.vertices(), graph.edges())
    ref = po.allpairs_topk(og, k, block=256)
    return t, og, ref


def _same(a, b, what):
    ai, ac, asc = a
    bi, bc, bsc = b
    assert np.array_equal(ai, bi), f"{what}: targets differ"
    assert np.array_equal(ac, bc), f"{what}: path counts differ"
    assert np.array_equal(asc.view(np.int64), bsc.view(np.int64)), f"{what}: score bits differ"


@pytest.fixture(scope="module")
def config3_10k():
    from dpathsim.synth import synth_config
    g = synth_config("config3", scale=0.01)
    t, og, ref = _typed_and_oracles(g, 100)
    return t, og, ref


@pytest.mark.parametrize("k", [10, 100])
@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_c_oracle_shortcuts_vs_numpy_config3_10k(config3_10k, k, flags):
    t, og, ref = config3_10k
    co = po.COracle.from_typed(t)
    assert co.n_authors == 10_000
    try:
        co.set_flags(flags)
        assert co.narrow() == (not (flags & po.COracle.FORCE_I64))   # int32 proof holds here
        got = co.topk(k, threads=4)
    finally:
        co.set_flags(0)
    # (score desc, ordinal asc) is a total order and the zero fill follows it, so
    # the top-k is the first k columns of the numpy top-100
    _same(got, tuple(a[:, :k] for a in ref), f"k={k} flags={flags}")


def test_c_oracle_wide_counts_vs_numpy():
    """A graph whose M needs int64 accumulators: few venues, prolific authors
    (C[x,v] in the thousands), so fits_i32 fails and the int64 path runs with
    the skip bound on and off."""
    from dpathsim.synth import synth_dblp
    g = synth_dblp(400, 600_000, 3, seed=7, author_alpha=1.1, authors_lambda=0.5)
    t, og, ref = _typed_and_oracles(g, 20)
    assert int(og.C.max()) > 1000
    co = po.COracle.from_typed(t)
    assert not co.narrow()
    m_max = int((og.C @ og.C.T).max())
    assert m_max >= 2 ** 31, m_max          # the counts really need 64 bits
    for flags in (0, po.COracle.NO_SKIP):
        try:
            co.set_flags(flags)
            _same(co.topk(20, threads=4), ref, f"wide flags={flags}")
        finally:
            co.set_flags(0)


def test_c_oracle_shortcuts_vs_numpy_config3_100k_rows():
    """config3 at 1/10 scale (100k authors, g up to 3.3e6): 300 random rows plus
    the 100 largest-g rows at k = 100, shortcuts on and forced off."""
    from dpathsim.graph import APVPA
    from dpathsim.synth import synth_config
    g = synth_config("config3", scale=0.1)
    og = po.OracleGraph(g.vertices(), g.edges())
    rng = np.random.default_rng(1)
    rows = np.unique(np.concatenate([rng.choice(len(og.authors), 300, replace=False),
                                     np.argsort(og.g)[-100:]]))
    ref = po.allpairs_topk(og, 100, rows=rows, block=100)
    co = po.COracle.from_typed(g.typed(APVPA))
    for flags in (0, po.COracle.FORCE_I64 | po.COracle.NO_SKIP):
        try:
            co.set_flags(flags)
            _same(co.topk_rows(100, rows, threads=4), ref, f"100k flags={flags}")
        finally:
            co.set_flags(0)
