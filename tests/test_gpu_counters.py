"""The lean hot kernel's work counters (workspace words 1-2), which the bench's
LDS roofline is priced from (bench.py), match the counts derived
on the host from the C^T tile layout."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _counts(eng):
    import torch
    w = eng.tensor("topk_ws")[:24].view(torch.int64).cpu().numpy()
    return int(w[1]), int(w[2])


@pytest.mark.parametrize("tile_w,half,npass", [(8192, False, 4), (16384, False, 8),
                                               (16384, True, 4), (7680, False, 4),
                                               (15360, False, 8), (15360, True, 4)])
def test_lean_counters_without_tile_skipping(tile_w, half, npass):
    """With tile skipping off every tile of every row is scanned with 32-bit
    counters: 4 passes of 2048 targets per 8192-target tile (W = 8192, and W =
    16384 whose unbounded tiles run as two u8 halves of the companion tiles),
    8 per 4-bit W = 16384 tile without companions.  So passes = npass * T * rows
    (d > 0), chunks = npass * sum_x sum_{v in x} (words of v over all tiles) / 4,
    T and the words those of the tile set the passes read."""
    from dpathsim.engine import PathSimEngine
    from dpathsim.synth import synth_dblp
    t = synth_dblp(40_000, 120_000, 500, seed=7).typed()
    eng = PathSimEngine(t, tile_w=tile_w)
    eng.half_tiles = half
    eng.venue_skip = False          # every bucket of the row's venues is scattered
    eng.upload().build()
    na, nv = t.n_authors, t.n_mids
    tw = tile_w // 2 if half else tile_w   # (the T15 widths 7680 / 15360 alike)
    T = (na + tw - 1) // tw
    cp = eng.tensor("c_ptr")[: na + 1].cpu().numpy()
    cc = eng.tensor("c_col")[: cp[-1]].cpu().numpy().astype(np.int64)
    off = eng.tensor("half_off" if half else "tile_off")[: nv * T + 1].cpu().numpy().astype(np.int64)
    off &= 0xFFFFFFFF
    words_v = off[(np.arange(nv) + 1) * T] - off[np.arange(nv) * T]
    assert (words_v % 4 == 0).all()
    rows_nonempty = int((np.diff(cp) > 0).sum())
    eng.tile_skip = False
    eng.topk(10, 0, na, heavy_first=False)
    n_pass, n_chunk = _counts(eng)
    assert n_pass == npass * T * rows_nonempty
    assert n_chunk == npass * int((words_v[cc] // 4).sum())
    # with tile skipping: fewer, and the same again on a re-run (counts are per launch)
    eng.tile_skip = True
    eng.topk(10, 0, na)
    a = _counts(eng)
    eng.topk(10, 0, na)
    b = _counts(eng)
    assert a == b
    assert 0 < a[0] < n_pass and 0 < a[1] < n_chunk
