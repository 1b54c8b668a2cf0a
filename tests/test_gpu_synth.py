"""GPU parity on seeded synthetic graphs: HIP path vs the C oracle, bit-exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _oracle(typed):
    import pathsim_oracle as po
    return po.COracle.from_typed(typed)


def _check(eng, co, k, rows=None):
    na = eng.typed.n_authors
    r0, r1 = (0, na) if rows is None else rows
    idx, cnt, sc = eng.topk(k, r0, r1)
    oi, oc, os_ = co.topk(k, r0, r1)
    gi, gc, gs = idx.cpu().numpy(), cnt.cpu().numpy(), sc.cpu().numpy()
    bad = np.flatnonzero((gi != oi).any(1) | (gc != oc).any(1) |
                         (gs.view(np.int64) != os_.view(np.int64)).any(1))
    assert len(bad) == 0, (f"{len(bad)} rows differ; first row {r0 + bad[0]}:\n"
                           f"gpu {gi[bad[0]]} {gc[bad[0]]} {gs[bad[0]]}\n"
                           f"orc {oi[bad[0]]} {oc[bad[0]]} {os_[bad[0]]}")


@pytest.mark.parametrize("tile_w", [256, 1024, 4096, 8192, 16384, 32768, 65536, 7680, 15360])
def test_synth_20k_top10(tile_w):
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_dblp
    g = synth_dblp(20_000, 60_000, 500, seed=7)
    t = g.typed()
    eng = build_engine(t, tile_w=tile_w)
    co = _oracle(t)
    cp, cc, cv, s, gg = co.export()
    nnz = eng.info.nnz_c
    assert np.array_equal(eng.tensor("c_ptr")[: t.n_authors + 1].cpu().numpy(), cp)
    assert np.array_equal(eng.tensor("c_col")[:nnz].cpu().numpy(), cc)
    assert np.array_equal(eng.tensor("c_val")[:nnz].cpu().numpy(), cv)
    assert np.array_equal(eng.tensor("g")[: t.n_authors].cpu().numpy(), gg)
    _check(eng, co, 10)


@pytest.mark.parametrize("tile_w,nw", [(8192, 1), (8192, 4), (4096, 4), (16384, 1), (32768, 1)])
def test_synth_20k_waves_per_row(tile_w, nw, tune):
    """Both kernel shapes -- one wave per row and a workgroup per row
    (dps_set_tuning overrides the tile-width default) -- give the oracle's top-k."""
    from dpathsim import _lib
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_dblp
    tune(_lib.TUNE_WAVES_PER_ROW, nw)
    t = synth_dblp(20_000, 60_000, 500, seed=7).typed()
    _check(build_engine(t, tile_w=tile_w), _oracle(t), 10)
    _check(build_engine(t, tile_w=tile_w), _oracle(t), 100, rows=(0, 3000))


@pytest.mark.parametrize("k", [1, 64, 65, 100, 200, 256])
def test_synth_k_variants(k):
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_dblp
    g = synth_dblp(3_000, 9_000, 200, seed=11)
    t = g.typed()
    _check(build_engine(t, tile_w=512), _oracle(t), k)


def test_heavy_rows_many_venues():
    """Rows with > 64 venues take the general (non-register) path."""
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_dblp
    g = synth_dblp(300, 40_000, 2_000, seed=5, mid_alpha=0.2, authors_lambda=6.0)
    t = g.typed()
    eng = build_engine(t, tile_w=256)
    d = np.diff(eng.tensor("c_ptr")[: t.n_authors + 1].cpu().numpy())
    assert d.max() > 64
    _check(eng, _oracle(t), 10)


def test_aptpa_multi_topic():
    from dpathsim.engine import build_engine
    from dpathsim.graph import APTPA
    from dpathsim.synth import synth_dblp
    g = synth_dblp(5_000, 15_000, 3_000, seed=3, metapath=APTPA)
    t = g.typed(APTPA)
    _check(build_engine(t, tile_w=1024), _oracle(t), 10)


@pytest.mark.parametrize("tile_w,glob", [(256, "0"), (1024, "0"), (8192, "0"), (8192, "1")])
def test_many_mids_tile_build(tile_w, glob, tune):
    """More mids than one block's LDS counters (20,000 venues > 8192): the
    block-local tile build with one block per mid range (default) and the
    global-atomic build (dps_set_tuning TILE_BUILD = 2) against the oracle."""
    from dpathsim import _lib
    tune(_lib.TUNE_TILE_BUILD, 2 if glob == "1" else 0)
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_dblp
    t = synth_dblp(6_000, 24_000, 20_000, seed=29).typed()
    assert t.n_mids > 2 * 8192
    _check(build_engine(t, tile_w=tile_w), _oracle(t), 10)


@pytest.mark.parametrize("tile_w", [16384, 32768])
def test_config3_sample_rows(tile_w):
    """Full-size config3 (1M authors): two 1500-row slices vs the C oracle."""
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_config
    g = synth_config("config3")
    t = g.typed()
    eng = build_engine(t, tile_w=tile_w)
    co = _oracle(t)
    _check(eng, co, 10, rows=(0, 1500))
    _check(eng, co, 10, rows=(777_000, 778_500))


def test_config4_aptpa_sample_rows():
    """Full-size config4 (APTPA, 200k topics, ~30 topics per row, rows > 64 topics
    take the general path): two 1000-row slices vs the C oracle."""
    from dpathsim.engine import build_engine
    from dpathsim.graph import APTPA
    from dpathsim.synth import synth_config
    t = synth_config("config4").typed(APTPA)
    eng = build_engine(t)
    co = _oracle(t)
    assert eng.info.nnz_c == len(co.export()[1])
    _check(eng, co, 10, rows=(0, 1000))
    _check(eng, co, 10, rows=(500_000, 501_000))


def test_config5_k100_sample_rows():
    """Full-size config5 (3M authors / 10M papers / 20k venues, top-100): two
    400-row slices vs the C oracle."""
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_config
    t = synth_config("config5").typed()
    eng = build_engine(t)
    co = _oracle(t)
    _check(eng, co, 100, rows=(0, 400))
    _check(eng, co, 100, rows=(2_999_600, 3_000_000))


@pytest.mark.parametrize("tile_w", [8192, 16384])
def test_bank_order_is_a_permutation(tile_w, tune):
    """dps_set_tuning BANK_ORDER = 1: every C^T bucket holds the
    same multiset of 16-bit entries, only ordered for the LDS banks, and the
    top-k is the oracle's."""
    from dpathsim import _lib
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_dblp
    t = synth_dblp(20_000, 60_000, 500, seed=7).typed()
    base = build_engine(t, tile_w=tile_w)
    tune(_lib.TUNE_BANK_ORDER, 1)
    eng = build_engine(t, tile_w=tile_w)
    off = base.tensor("tile_off").cpu().numpy().astype(np.int64)
    assert np.array_equal(off, eng.tensor("tile_off").cpu().numpy().astype(np.int64))
    n = int(off[-1]) * 2
    a = base.tensor("tile_ent").cpu().numpy().view(np.uint16)[:n]
    b = eng.tensor("tile_ent").cpu().numpy().view(np.uint16)[:n]
    bucket = np.repeat(np.arange(len(off) - 1), 2 * np.diff(off))
    ka = np.lexsort((a, bucket))
    kb = np.lexsort((b, bucket))
    assert np.array_equal(a[ka], b[kb])          # same entries per bucket
    assert not np.array_equal(a, b)              # ... in a different order
    _check(eng, _oracle(t), 10)


@pytest.mark.parametrize("tile_w", [1024, 8192, 16384, 32768])
def test_sorted_tile_build_matches_atomic(tile_w, tune):
    """dps_ct_tiles_build2's sorted layout (many mids: one radix sort of
    (bucket, entry) pairs) against dps_ct_tiles_build's global-atomic counting
    sort on the same C: identical offsets, maxima and tile minima, the same
    multiset of entries in every bucket (order inside a bucket is free), and
    the engine's top-k against the oracle."""
    import torch
    from dpathsim import _lib
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_dblp
    tune(_lib.TUNE_TILE_BUILD, 2)
    t = synth_dblp(6_000, 24_000, 20_000, seed=31).typed()
    eng = build_engine(t, tile_w=tile_w)
    d = eng._dev
    NA, NV = t.n_authors, t.n_mids
    T = (NA + tile_w - 1) // tile_w
    off = torch.empty(NV * T + 1, dtype=torch.int32, device=eng.device)
    mx = torch.empty_like(off)
    gm = torch.empty(T, dtype=torch.int64, device=eng.device)
    ent = torch.empty_like(d["tile_ent"])
    st = torch.zeros(1, dtype=torch.int32, device=eng.device)
    ws = torch.empty(_lib.size("dps_ct_tiles_workspace_size", NV, NA, tile_w), dtype=torch.uint8,
                     device=eng.device)
    _lib.call("dps_ct_tiles_build", d["c_ptr"].data_ptr(), d["c_col"].data_ptr(),
              d["c_val"].data_ptr(), d["den"].data_ptr(), d["t_rank"].data_ptr(), NA, NV, tile_w,
              off.data_ptr(), ent.data_ptr(), mx.data_ptr(), gm.data_ptr(), st.data_ptr(),
              ws.data_ptr(), ws.numel(), eng.stream)
    torch.cuda.synchronize()
    o1 = off.cpu().numpy().astype(np.int64)
    o2 = d["tile_off"].cpu().numpy().astype(np.int64)
    assert np.array_equal(o1, o2)
    assert np.array_equal(mx.cpu().numpy(), d["tile_maxc"].cpu().numpy()[: NV * T + 1])
    assert np.array_equal(gm.cpu().numpy(), d["tile_gmin"].cpu().numpy()[:T])
    per = 2 if tile_w <= 16384 else 1
    n = int(o1[-1]) * per
    view = (lambda a: a.view(np.uint16)) if per == 2 else (lambda a: a)
    a = view(ent.cpu().numpy())[:n]
    b = view(d["tile_ent"].cpu().numpy())[:n]
    bucket = np.repeat(np.arange(len(o1) - 1), per * np.diff(o1))
    assert np.array_equal(a[np.lexsort((a, bucket))], b[np.lexsort((b, bucket))])
    _check(eng, _oracle(t), 10)
