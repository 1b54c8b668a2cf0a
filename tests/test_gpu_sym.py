"""Symmetric mode (dps_cct_sym): each pair scanned once, records
handed to the other row, merged exactly -- against the C oracle and the
ordinary launch, bit for bit (idx, count, score bits).  (On config3 its output
digest equals the ordinary launch's, tools/ab_sym.py, profiles/r03/sym.)"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _np(o):
    return [a.cpu().numpy() for a in o]


def _same(a, b, what):
    bad = np.flatnonzero((a[0] != b[0]).any(1) | (a[1] != b[1]).any(1) |
                         (a[2].view(np.int64) != b[2].view(np.int64)).any(1))
    assert len(bad) == 0, (f"{what}: {len(bad)} rows differ; first row {bad[0]}:\n"
                           f"{a[0][bad[0]]} {a[1][bad[0]]} {a[2][bad[0]]}\n"
                           f"{b[0][bad[0]]} {b[1][bad[0]]} {b[2][bad[0]]}")


@pytest.mark.parametrize("tile_w", [8192, 16384])
@pytest.mark.parametrize("k", [10, 100])
def test_sym_synth_100k(tile_w, k):
    import pathsim_oracle as po
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_dblp
    t = synth_dblp(100_000, 300_000, 2_000, seed=13).typed()
    eng = build_engine(t, tile_w=tile_w, venue_skip=False)
    plain = _np(eng.topk(k))
    eng.sym = True
    got = _np(eng.topk(k))
    n_rec = eng.check_sym()
    assert n_rec > 0                                 # records were handed on
    _same(got, plain, "sym vs plain")
    want = po.COracle.from_typed(t).topk(k, 0, t.n_authors)
    _same(got, want, "sym vs oracle")
    kc = eng.kernel_counts()
    assert kc["passes"] > 0 and kc["chunks"] > 0


@pytest.mark.parametrize("band", [0, 2])
def test_sym_band_widths_and_capacity_rerun(band):
    """Other band widths; a record capacity far too small reruns with room."""
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_dblp
    t = synth_dblp(60_000, 180_000, 800, seed=17).typed()
    eng = build_engine(t, tile_w=8192, venue_skip=False)
    plain = _np(eng.topk(10))
    eng.sym, eng.sym_band, eng.sym_rec_per_row = True, band, 1e-4
    got = _np(eng.topk(10))
    _same(got, plain, f"sym band {band}")
    assert eng._sym_stat[1] > 6                       # the rerun's capacity


def test_sym_weak_rows_and_zero_fill():
    """Rows whose band holds fewer than k positive scores scan everything
    themselves (zero-score fill in reference order): a sparse graph."""
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_dblp
    t = synth_dblp(40_000, 20_000, 3_000, seed=19).typed()
    eng = build_engine(t, tile_w=8192, venue_skip=False)
    plain = _np(eng.topk(10))
    eng.sym = True
    got = _np(eng.topk(10))
    _same(got, plain, "sparse")
    assert (got[2][:, -1] == 0).any()                # some rows end in zero fill
