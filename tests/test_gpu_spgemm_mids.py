"""Single-mid SpGEMM edge cases against the C oracle: papers without a venue
inside long author rows (the LDS-histogram path of rows > 64 entries puts the
"no mid" bin last and drops it), duplicate authorships, and a mid count above
the histogram range (the sorting path)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _graph(n_mids, seed):
    from dpathsim.graph import Graph
    from dpathsim.synth import synth_dblp
    g = synth_dblp(20_000, 60_000, n_mids, seed=seed)
    rng = np.random.default_rng(seed)
    px = g.edge_rel_idx == 1
    keep = ~px | (rng.random(len(px)) > 0.3)          # 30 % of papers lose their venue
    src, dst, rel = g.edge_src[keep], g.edge_dst[keep], g.edge_rel_idx[keep]
    ap = np.flatnonzero(rel == 0)
    dup = rng.choice(ap, size=len(ap) // 10, replace=False)   # repeated authorships
    src = np.concatenate([src, src[dup]])
    dst = np.concatenate([dst, dst[dup]])
    rel = np.concatenate([rel, rel[dup]])
    return Graph(g.node_type_idx, g.type_names, src, dst, rel, g.rel_names)


@pytest.mark.parametrize("n_mids", [500, 10_000])
def test_single_mid_spgemm_long_rows(n_mids):
    import pathsim_oracle as po
    from dpathsim.engine import build_engine
    t = _graph(n_mids, 5).typed()
    eng = build_engine(t, tile_w=8192)
    assert eng.bounds.max_mids_per_paper <= 1             # the single-mid path runs
    co = po.COracle.from_typed(t)
    cp, cc, cv, s, gg = co.export()
    na = t.n_authors
    assert int(np.diff(cp[: na + 1]).max()) > 64           # long rows exist
    nnz = int(cp[na])
    assert np.array_equal(eng.tensor("c_ptr")[: na + 1].cpu().numpy(), cp[: na + 1])
    assert np.array_equal(eng.tensor("c_col")[:nnz].cpu().numpy(), cc[:nnz])
    assert np.array_equal(eng.tensor("c_val")[:nnz].cpu().numpy(), cv[:nnz])
    assert np.array_equal(eng.tensor("g")[:na].cpu().numpy(), gg[:na])
    idx, cnt, sc = eng.topk(10, 0, 4000)
    oi, oc, os_ = co.topk(10, 0, 4000)
    assert np.array_equal(idx.cpu().numpy(), oi)
    assert np.array_equal(cnt.cpu().numpy(), oc)
    assert np.array_equal(sc.cpu().numpy().view(np.int64), os_.view(np.int64))
