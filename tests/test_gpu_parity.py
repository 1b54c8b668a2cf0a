"""GPU parity: HIP path vs the oracle, bit-exact (gpu marker)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def small_engine(dblp_small_tuples):
    from dpathsim.graph import Graph
    from dpathsim.engine import build_engine
    v, e = dblp_small_tuples
    g = Graph.from_tuples(v, e)
    return build_engine(g.typed(), tile_w=256)


def test_dblp_small_counts_bit_exact(small_engine, dblp_small_expected):
    eng = small_engine
    ex = dblp_small_expected
    nnz = eng.info.nnz_c
    assert nnz == len(ex["c_col"])
    assert np.array_equal(eng.tensor("c_ptr")[: len(ex["c_ptr"])].cpu().numpy(), ex["c_ptr"])
    assert np.array_equal(eng.tensor("c_col")[:nnz].cpu().numpy(), ex["c_col"])
    assert np.array_equal(eng.tensor("c_val")[:nnz].cpu().numpy(), ex["c_val"])
    assert np.array_equal(eng.tensor("s")[: len(ex["s"])].cpu().numpy(), ex["s"])
    assert np.array_equal(eng.tensor("g")[: len(ex["g"])].cpu().numpy(), ex["g"])


@pytest.mark.parametrize("tile_w", [256, 512, 4096, 16384, 7680, 15360])
def test_dblp_small_top10_bit_exact(dblp_small_tuples, dblp_small_expected, tile_w):
    from dpathsim.graph import Graph
    from dpathsim.engine import build_engine
    v, e = dblp_small_tuples
    eng = build_engine(Graph.from_tuples(v, e).typed(), tile_w=tile_w)
    idx, cnt, sc = eng.topk(10)
    ex = dblp_small_expected
    assert np.array_equal(idx.cpu().numpy(), ex["top10_idx"])
    assert np.array_equal(cnt.cpu().numpy(), ex["top10_cnt"])
    assert np.array_equal(sc.cpu().numpy().view(np.int64), ex["top10_score"].view(np.int64))


def test_target_order_is_stable_g_sort(small_engine):
    eng = small_engine
    g = eng.tensor("g")[: eng.n_targets].cpu().numpy()
    perm = eng.tensor("t_perm")[: eng.n_targets].cpu().numpy()
    rank = eng.tensor("t_rank")[: eng.n_targets].cpu().numpy()
    g_t = eng.tensor("g_t")[: eng.n_targets].cpu().numpy()
    expect = np.lexsort((np.arange(len(g)), g))
    assert np.array_equal(perm, expect)
    assert np.array_equal(rank[perm], np.arange(len(g)))
    assert np.array_equal(g_t, g[perm])


def test_tile_skip_does_not_change_results(dblp_small_tuples, dblp_small_expected):
    from dpathsim.graph import Graph
    from dpathsim.engine import build_engine
    v, e = dblp_small_tuples
    eng = build_engine(Graph.from_tuples(v, e).typed(), tile_w=256)
    eng.tile_skip = False
    idx, cnt, sc = eng.topk(10)
    ex = dblp_small_expected
    assert np.array_equal(idx.cpu().numpy(), ex["top10_idx"])
    assert np.array_equal(sc.cpu().numpy().view(np.int64), ex["top10_score"].view(np.int64))


@pytest.mark.parametrize("tile_w", [256, 8192, 16384, 65536, 7680, 15360])
def test_single_source_walks_match_oracle(dblp_small_tuples, tile_w):
    """dps_walk_row / dps_pair_count / global walk; W = 65536 runs walk_row in
    two 32768-label parts."""
    import pathsim_oracle as po
    from dpathsim.engine import build_engine
    from dpathsim.graph import Graph
    v, e = dblp_small_tuples
    og = po.OracleGraph(v, e)
    eng = build_engine(Graph.from_tuples(v, e).typed(), tile_w=tile_w)
    t = eng.typed
    graph = t.graph
    rng = np.random.default_rng(1)
    nodes = list(rng.choice(graph.n_nodes, 25, replace=False)) + [int(t.author_nodes[0])]
    M = (og.C @ og.C.T).toarray()
    for n in nodes:
        nid = graph.node_id(int(n))
        assert eng.global_walk(int(n)) == og.global_walk(nid)
        row = eng.walk_row(int(n)).cpu().numpy()
        expect = np.array([og.pairwise_walk(nid, a) for a in og.authors])
        assert np.array_equal(row, expect), nid
    for a, b in rng.choice(len(og.authors), (30, 2)):
        na_, nb_ = int(t.author_nodes[a]), int(t.author_nodes[b])
        assert eng.pairwise_walk(na_, nb_) == M[a, b]
