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
