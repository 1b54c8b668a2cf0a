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
