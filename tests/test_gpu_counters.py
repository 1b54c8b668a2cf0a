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


def test_lean_counters_without_tile_skipping():
    """With tile skipping off every tile of every row is scanned with four
    32-bit passes: passes = 4 T * rows(d > 0), chunks = 4 * sum_x sum_{v in x}
    (entries of v over all tiles) / 4 words."""
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_dblp
    t = synth_dblp(20_000, 60_000, 500, seed=7).typed()
    eng = build_engine(t, tile_w=8192)
    na, nv = t.n_authors, t.n_mids
    T = (na + 8191) // 8192
    cp = eng.tensor("c_ptr")[: na + 1].cpu().numpy()
    cc = eng.tensor("c_col")[: cp[-1]].cpu().numpy().astype(np.int64)
    off = eng.tensor("tile_off")[: nv * T + 1].cpu().numpy().astype(np.int64) & 0xFFFFFFFF
    words_v = off[(np.arange(nv) + 1) * T] - off[np.arange(nv) * T]
    assert (words_v % 4 == 0).all()
    rows_nonempty = int((np.diff(cp) > 0).sum())
    eng.tile_skip = False
    eng.topk(10, 0, na, heavy_first=False)
    n_pass, n_chunk = _counts(eng)
    assert n_pass == 4 * T * rows_nonempty
    assert n_chunk == 4 * int((words_v[cc] // 4).sum())
    # with tile skipping: fewer, and the same again on a re-run (counts are per launch)
    eng.tile_skip = True
    eng.topk(10, 0, na)
    a = _counts(eng)
    eng.topk(10, 0, na)
    b = _counts(eng)
    assert a == b
    assert 0 < a[0] < n_pass and 0 < a[1] < n_chunk
