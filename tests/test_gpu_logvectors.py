"""GPU: the reference's own logged operands through the device score division.

The 2018 run log (output/d_pathsim_output_20180417_020445.log:1-406, copied as
data into tests/golden/log_triples.json by make_golden.py) holds 81 stages of
(pairwise walk pw, target global walk gy, score) for the source 'Jiawei Han'
(gx = 8423).  Each (pw, gy) goes through dps_row_scores -- the same
`(double)(2*m) / (double)(gx + g)` the hot kernel applies (DPathSim_APVPA.py:51-52)
-- and the repr of every device score must equal the logged score string.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_logged_triples_through_device_scores(log_triples):
    import torch
    from dpathsim import _lib

    _lib.load()
    gx = int(log_triples["source_global_walk"])
    st = log_triples["stages"]
    assert len(st) == 81 and gx == 8423
    m = torch.tensor([s["pw"] for s in st], dtype=torch.int64, device="cuda")
    g = torch.tensor([s["gy"] for s in st], dtype=torch.int64, device="cuda")
    out = torch.empty(len(st), dtype=torch.float64, device="cuda")
    zd = torch.zeros(1, dtype=torch.int64, device="cuda")
    _lib.call("dps_row_scores", m.data_ptr(), g.data_ptr(), gx, len(st), out.data_ptr(),
              zd.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    assert int(zd.item()) == 0
    assert [repr(float(v)) for v in got] == [s["score_repr"] for s in st]
    # and bit for bit against Python's int / int (the reference's arithmetic)
    expect = np.array([2 * s["pw"] / (gx + s["gy"]) for s in st], dtype=np.float64)
    assert np.array_equal(got.view(np.int64), expect.view(np.int64))
    # the log's denominators are far larger than dblp_small's (g <= 1396)
    assert max(gx + s["gy"] for s in st) > 8423
