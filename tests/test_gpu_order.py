"""The heavy-first dequeue list (dps_heavy_first): a stable descending order of
the rows by their work on a log scale (four steps per octave), the first
n_split rows repeated `pieces` times in front."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _key(w):
    out = np.empty(len(w), dtype=np.int64)
    for i, x in enumerate(w.tolist()):
        b = 0
        if x > 0:
            e = x.bit_length() - 1
            b = 1 + 4 * e + (((x << (63 - e)) >> 61) & 3)
        out[i] = 255 - b
    return out


@pytest.mark.parametrize("n,row_begin,n_split,pieces", [(1, 0, 0, 1), (5000, 0, 0, 1),
                                                        (100_000, 3, 256, 16), (70_001, 100, 7, 3)])
def test_heavy_first_order(n, row_begin, n_split, pieces):
    import torch
    from dpathsim import _lib
    rng = np.random.default_rng(n)
    w = (rng.pareto(1.2, n) * 1000).astype(np.int64)
    w[rng.integers(0, n, n // 10)] = 0
    if n >= 3:
        w[:3] = [2**40 + 5, 2**33, 1]
    wt = torch.from_numpy(w).cuda()
    dq = torch.empty(n + n_split * (pieces - 1), dtype=torch.int32, device="cuda")
    ws = torch.empty(max(_lib.size("dps_heavy_first_workspace_size", n), 256), dtype=torch.uint8,
                     device="cuda")
    _lib.call("dps_heavy_first", wt.data_ptr(), n, row_begin, n_split, pieces, dq.data_ptr(),
              ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream)
    got = dq.cpu().numpy().astype(np.int64) - row_begin
    expect = np.argsort(_key(w), kind="stable")
    assert np.array_equal(got[n_split * pieces:], expect[n_split:])
    assert np.array_equal(got[:n_split * pieces], np.repeat(expect[:n_split], pieces))


def _hv_host(n_v, n_hv):
    """smallest thr >= 1 with |{v : n_v >= thr}| <= n_hv; slots in venue order"""
    a = np.sort(n_v.astype(np.int64))[::-1]
    thr = 1 if len(a) <= n_hv else max(1, int(a[n_hv]) + 1)
    heavy = n_v.astype(np.int64) >= thr
    slot = np.full(len(n_v), -1, dtype=np.int64)
    slot[heavy] = np.arange(int(heavy.sum()))
    return slot


@pytest.mark.parametrize("n,n_hv,kind", [(1, 32, "rand"), (31, 32, "rand"), (32, 32, "rand"),
                                         (33, 32, "rand"), (5000, 32, "rand"), (5000, 1, "ties"),
                                         (5000, 64, "ties"), (200_000, 32, "rand"),
                                         (70_001, 17, "big"), (4096, 32, "zeros")])
def test_heavy_venues_select(n, n_hv, kind):
    """dps_heavy_venues (radix select since round 6) against the host rule."""
    import torch
    from dpathsim import _lib
    rng = np.random.default_rng(n + n_hv)
    if kind == "rand":
        v = (rng.pareto(1.1, n) * 50).astype(np.uint32)
    elif kind == "ties":
        v = rng.integers(0, 6, n).astype(np.uint32)
    elif kind == "big":
        v = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        v[:5] = 2**32 - 1
    else:
        v = np.zeros(n, np.uint32)
        v[rng.integers(0, n, 10)] = rng.integers(1, 100, 10).astype(np.uint32)
    vt = torch.from_numpy(v.view(np.int32)).cuda()
    slot = torch.full((n,), -7, dtype=torch.int32, device="cuda")
    _lib.call("dps_heavy_venues", vt.data_ptr(), n, n_hv, slot.data_ptr(),
              torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = slot.cpu().numpy().astype(np.int64)
    assert np.array_equal(got, _hv_host(v, n_hv))
    assert (got >= 0).sum() <= n_hv
