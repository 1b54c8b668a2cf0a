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
    assert np.array_equal(eng.tensor("c_ptr").cpu().numpy(), ex["c_ptr"])
    assert np.array_equal(eng.tensor("c_col")[:nnz].cpu().numpy(), ex["c_col"])
    assert np.array_equal(eng.tensor("c_val")[:nnz].cpu().numpy(), ex["c_val"])
    assert np.array_equal(eng.tensor("s")[: len(ex["s"])].cpu().numpy(), ex["s"])
    assert np.array_equal(eng.tensor("g")[: len(ex["g"])].cpu().numpy(), ex["g"])


@pytest.mark.parametrize("tile_w", [256, 512, 4096])
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
