"""The fused walk pass of the build (dps_walks_fused: s, n_v, g, diag, row work
in two passes over C) against the separate entry points and the C oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n_mids", [500, 20_000, 40_000])
def test_fused_walks_match_separate_entry_points(n_mids):
    """500 mids: the LDS column sums of one range; 20k / 40k: mids over several
    12288-mid LDS ranges, the last one partial -- the engine's bucketed column
    sums (dps_walks_fused_ws) and the per-range re-reading kernel
    (dps_walks_fused without a workspace) must agree with each other and the
    oracle."""
    import torch
    import pathsim_oracle as po
    from dpathsim import _lib
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_dblp
    t = synth_dblp(20_000, 60_000, n_mids, seed=13).typed()
    eng = build_engine(t)
    co = po.COracle.from_typed(t)
    cp, cc, cv, s_o, g_o = co.export()
    na, nv, nr = t.n_authors, t.n_mids, t.n_rows
    d = eng._dev
    assert np.array_equal(d["s"][:nv].cpu().numpy(), s_o[:nv])
    assert np.array_equal(d["g"][:na].cpu().numpy(), g_o[:na])
    st = torch.cuda.current_stream().cuda_stream
    s = torch.empty(nv, dtype=torch.int64, device="cuda")
    _lib.call("dps_col_sums", d["c_ptr"].data_ptr(), d["c_col"].data_ptr(), d["c_val"].data_ptr(),
              nr, nv, s.data_ptr(), st)
    terms = torch.empty(na, dtype=torch.int64, device="cuda")
    ncol = torch.empty(nv, dtype=torch.int32, device="cuda")
    _lib.call("dps_row_work", d["c_ptr"].data_ptr(), d["c_col"].data_ptr(), na, nv,
              ncol.data_ptr(), terms.data_ptr(), st)
    assert torch.equal(s, d["s"][:nv])
    assert torch.equal(terms, d["row_terms"][:na])   # the fused pass's n_v (author entries per mid)
    # row work = sum over the row's venues of the author entries per venue
    n_v = np.bincount(cc[: cp[na]], minlength=nv)
    expect = np.add.reduceat(n_v[cc[: cp[na]]], cp[:na]) * (np.diff(cp[: na + 1]) > 0)
    assert np.array_equal(terms.cpu().numpy(), expect)
    # the same pass without a workspace (per-range re-reads for wide mids)
    s2 = torch.empty(nv, dtype=torch.int64, device="cuda")
    nv2 = torch.empty(nv, dtype=torch.int32, device="cuda")
    g2 = torch.empty(na, dtype=torch.int64, device="cuda")
    t2 = torch.empty(na, dtype=torch.int64, device="cuda")
    _lib.call("dps_walks_fused", d["c_ptr"].data_ptr(), d["c_col"].data_ptr(), d["c_val"].data_ptr(),
              nr, na, nv, s2.data_ptr(), nv2.data_ptr(), g2.data_ptr(), None, t2.data_ptr(), None, st)
    assert torch.equal(s2, d["s"][:nv])
    assert torch.equal(g2, d["g"][:na])
    assert torch.equal(t2, d["row_terms"][:na])
    assert np.array_equal(nv2.cpu().numpy(), n_v)
