"""Venue skipping (dps_venue_skip) against the C oracle and
against the same kernel without it: bit-exact top-k (idx, count, score bits).

Venue skipping stops scattering a heavy venue's C^T buckets once the row's
k-th score makes the venue unable to lift a target to the top-k on its own,
and completes every flagged target's count from the dense heavy-venue table.
These tests pin that the pruning is exact, that it actually fires (the
kernel's counter of table-completed candidates), and that it composes with
the split-row pieces, k > 64 (two top-k registers per lane), rows with more
than 64 venues and the u16 / u32 accumulator passes.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _np(t):
    return [a.cpu().numpy() for a in t]


def _same(got, want, r0=0):
    gi, gc, gs = got
    oi, oc, os_ = want
    bad = np.flatnonzero((gi != oi).any(1) | (gc != oc).any(1) |
                         (gs.view(np.int64) != os_.view(np.int64)).any(1))
    assert len(bad) == 0, (f"{len(bad)} rows differ; first row {r0 + bad[0]}:\n"
                           f"got  {gi[bad[0]]} {gc[bad[0]]} {gs[bad[0]]}\n"
                           f"want {oi[bad[0]]} {oc[bad[0]]} {os_[bad[0]]}")


def _pair(t, tile_w=8192, **kw):
    from dpathsim.engine import build_engine
    on = build_engine(t, tile_w=tile_w, venue_skip=True, **kw)
    off = build_engine(t, tile_w=tile_w, venue_skip=False, **kw)
    assert on._ext is not None and on._ext.s and (off._ext is None or not off._ext.s)
    return on, off


@pytest.mark.parametrize("tile_w", [8192, 16384])
@pytest.mark.parametrize("k", [10, 100])
def test_venue_skip_synth_exact_and_fires(k, tile_w):
    import pathsim_oracle as po
    from dpathsim.synth import synth_dblp
    t = synth_dblp(60_000, 180_000, 800, seed=13).typed()
    on, off = _pair(t, tile_w)
    got = _np(on.topk(k, heavy_first=False))
    cnt = on.kernel_counts()
    ref = _np(off.topk(k, heavy_first=False))
    cnt_off = off.kernel_counts()
    _same(got, ref)
    co = po.COracle.from_typed(t)
    _same(got, co.topk(k, 0, t.n_authors))
    print(f"k={k}: with venue skipping {cnt}, without {cnt_off}")
    assert cnt["verified"] > 0 and cnt_off["verified"] == 0
    assert cnt["chunks"] < cnt_off["chunks"]


@pytest.mark.parametrize("tile_w", [8192, 16384])
def test_venue_skip_split_pieces_and_wide_rows(tile_w):
    """The bench entry point (heavy-first, split pieces + merge) on a graph with
    rows of > 64 venues and heavily shared venues (large counts)."""
    import pathsim_oracle as po
    from dpathsim.synth import synth_dblp
    t = synth_dblp(40_000, 200_000, 3_000, seed=21, mid_alpha=1.1, authors_lambda=3.0).typed()
    on, off = _pair(t, tile_w)
    d = np.diff(on.tensor("c_ptr")[: t.n_authors + 1].cpu().numpy())
    assert d.max() > 64
    got = _np(on.topk(10, split_rows=64, pieces=4))
    _same(got, _np(off.topk(10, split_rows=64, pieces=4)))
    co = po.COracle.from_typed(t)
    _same(got, co.topk(10, 0, t.n_authors))
    assert on.kernel_counts()["verified"] > 0


def test_venue_skip_row_list_and_slices():
    """dps_cct_topk_rows and row sub-ranges take the same pruning."""
    import pathsim_oracle as po
    from dpathsim.synth import synth_dblp
    t = synth_dblp(30_000, 90_000, 400, seed=5).typed()
    on, _ = _pair(t)
    co = po.COracle.from_typed(t)
    rows = np.random.default_rng(3).choice(t.n_authors, 4000, replace=False)
    _same(_np(on.topk_rows(10, rows)), co.topk_rows(10, rows))
    _same(_np(on.topk(10, 1000, 9000)), co.topk(10, 1000, 9000), 1000)


def test_venue_skip_diag_denominator_is_off():
    """The pruning needs g = C.s; the diag denominator builds no table."""
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_dblp
    t = synth_dblp(5_000, 15_000, 200, seed=2).typed()
    eng = build_engine(t, tile_w=8192, denominator="diag")
    assert (eng._ext is None or not eng._ext.s) and eng.tensor("hv_c") is None


@pytest.mark.parametrize("n_hv,perm,n", [(32, True, 50_000), (32, False, 3), (31, True, 20_000),
                                         (64, True, 20_000), (2, True, 1000)])
def test_heavy_table_against_host(n_hv, perm, n):
    """dps_heavy_table (whole rows for n_hv = 32 / 64 since round 6, the scattered
    2-byte form otherwise) against the dense table built on the host: rows
    with up to 300 venues, counts above 65535 saturated, labels permuted."""
    import torch
    from dpathsim import _lib
    rng = np.random.default_rng(n_hv * 7 + n)
    nv = 4000
    deg = np.minimum(rng.geometric(0.15, n), 300)
    deg[: min(3, n)] = [300, 0, 1][: min(3, n)]
    ptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    col = np.concatenate([np.sort(rng.choice(nv, d, replace=False)) for d in deg]).astype(np.int32)
    val = rng.integers(1, 200, len(col)).astype(np.int32)
    val[:5] = [70000, 65535, 65534, 1, 2**31 - 1][: len(val[:5])]
    n_v = np.bincount(col, minlength=nv).astype(np.uint32)
    ranks = rng.permutation(n).astype(np.int32) if perm else None
    dev = "cuda"
    tt = lambda a: torch.from_numpy(a).to(dev)   # noqa: E731
    # (device copies held in names until the kernels have run: a temporary's
    # memory goes back to the caching allocator as soon as data_ptr() returns)
    nv_d, ptr_d, col_d, val_d = tt(n_v.view(np.int32)), tt(ptr), tt(col), tt(val)
    rk = tt(ranks) if perm else None
    slot = torch.empty(nv, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    _lib.call("dps_heavy_venues", nv_d.data_ptr(), nv, n_hv, slot.data_ptr(), st)
    hv = torch.full((n * n_hv,), 0x5A5A, dtype=torch.int16, device=dev)   # garbage: rows are written whole
    _lib.call("dps_heavy_table", ptr_d.data_ptr(), col_d.data_ptr(), val_d.data_ptr(),
              rk.data_ptr() if perm else None, n, slot.data_ptr(), n_hv, hv.data_ptr(), st)
    torch.cuda.synchronize()
    got = hv.cpu().numpy().view(np.uint16).reshape(n, n_hv)
    sl = slot.cpu().numpy()
    want = np.zeros((n, n_hv), np.uint16)
    row = np.repeat(np.arange(n), deg)
    lab = ranks[row] if perm else row
    h = sl[col] >= 0
    want[lab[h], sl[col][h]] = np.minimum(val[h], 0xFFFF).astype(np.uint16)
    assert np.array_equal(got, want)
