"""The T15 tile layout (round 6; dps_cct1.hip Geo, include/dpathsim.h): tiles of
15360 targets in 4-bit counters (companion u8 halves of 7680) or 7680 in u8,
whose 7680-byte accumulators keep 20 one-wave workgroups resident per CU where
8 KiB keeps 18.  Every build path (block-local over one and several mid
ranges, the global-atomic and the sorted builds) and kernel path (u8 / 4-bit
base passes, split rows, the wide u16 / u32 passes elsewhere in
test_gpu_fullsize) against the oracle, and the same lists as the power-of-two
tiles."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _cmp(got, want):
    gi, gc, gs = (a.cpu().numpy() for a in got)
    oi, oc, os_ = want
    bad = np.flatnonzero((gi != oi).any(1) | (gc != oc).any(1) |
                         (gs.view(np.int64) != os_.view(np.int64)).any(1))
    assert len(bad) == 0, (f"{len(bad)} rows differ; first row {bad[0]}:\n"
                           f"gpu {gi[bad[0]]} {gc[bad[0]]} {gs[bad[0]]}\n"
                           f"orc {oi[bad[0]]} {oc[bad[0]]} {os_[bad[0]]}")


@pytest.mark.parametrize("tile_w", [7680, 15360])
@pytest.mark.parametrize("build", [1, 2])
def test_t15_many_mids_both_builds(tile_w, build, tune):
    """20k venues: the block-local build over three mid ranges (1) and the
    global-atomic build (2); k = 10 and 100."""
    import pathsim_oracle as po
    from dpathsim import _lib
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_dblp
    tune(_lib.TUNE_TILE_BUILD, build)
    t = synth_dblp(70_000, 200_000, 20_000, seed=31).typed()
    eng = build_engine(t, tile_w=tile_w)
    co = po.COracle.from_typed(t)
    for k in (10, 100):
        _cmp(eng.topk(k), co.topk(k, 0, t.n_authors))


def test_t15_sorted_build_config4_shape():
    """APTPA at 5 % of config4 (10k topics, several per paper): more mid ranges
    than the block-local build takes, so the sorted build (dps_ct_tiles_build2)
    runs, at 7680 (u8) and 15360 (4-bit)."""
    import pathsim_oracle as po
    import dpathsim
    from dpathsim.engine import build_engine
    from dpathsim.synth import CONFIGS, synth_config
    t = synth_config("config4", scale=0.05).typed(dpathsim.METAPATHS[CONFIGS["config4"][3]])
    co = po.COracle.from_typed(t)
    want = co.topk(10, 0, t.n_authors)
    for w in (7680, 15360):
        _cmp(build_engine(t, tile_w=w).topk(10), want)


def test_t15_equals_power_of_two_tiles():
    """The tile width is a layout choice: 15360 / 7680 give the lists of 16384 /
    8192 on a 100k-author graph (bench-shaped: venue skipping, companion tiles,
    split heavy rows)."""
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_config
    t = synth_config("config3_100k").typed()
    for a, b in ((16384, 15360), (8192, 7680)):
        ga = [x.cpu().numpy() for x in build_engine(t, tile_w=a).topk(10)]
        gb = [x.cpu().numpy() for x in build_engine(t, tile_w=b).topk(10)]
        for x, y in zip(ga, gb):
            assert np.array_equal(x.view(np.int64) if x.dtype == np.float64 else x,
                                  y.view(np.int64) if y.dtype == np.float64 else y), (a, b)


def test_t15_engine_keeps_sym_to_power_of_two_widths():
    """The symmetric mode has no T15 form: at 15360 the engine runs the ordinary
    launch (same lists as without sym)."""
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_dblp
    t = synth_dblp(6_000, 18_000, 300, seed=13).typed()
    eng = build_engine(t, tile_w=15360)
    eng.sym = True
    a = [x.cpu().numpy() for x in eng.topk(10)]
    eng.sym = False
    b = [x.cpu().numpy() for x in eng.topk(10)]
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
