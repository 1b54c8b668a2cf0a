"""A8 log format (DPathSim_APVPA.py:32-67): the native all-pairs log writer and
its Python-repr float formatter, checked against Python's own formatting.
Host-only code: runs without a GPU."""
import math
import struct

import numpy as np
import pytest


def _fmt():
    from dpathsim.logfmt import format_float
    return format_float


EDGE = [0.0, 1.0, 0.5, 0.1, 1 / 3, 2 / 3, 1e-4, 9.999999999999999e-05, 1e-5, 1.5e-07, 1e16,
        9999999999999998.0, 1e15, 123456789012345678.0, 1e22, 1e-300, 5e-324, 2.2250738585072014e-308,
        1.7976931348623157e308, 0.30000000000000004, 100.0, 12345.678, 6.1349693251533744e-06,
        0.0001, 0.00011, 1e-4 * (1 - 2 ** -52), 2.0 ** -1074, 2.0 ** 60, 3.0e-05, -0.25, -1e-7]


def test_format_float_edge_cases():
    f = _fmt()
    for v in EDGE:
        assert f(v) == repr(v), v


def test_format_float_random_bits_and_scores():
    f = _fmt()
    rng = np.random.default_rng(5)
    bits = rng.integers(0, 2 ** 63 - 1, size=3000, dtype=np.int64)
    for b in bits:
        v = struct.unpack("<d", struct.pack("<q", int(b)))[0]
        if math.isfinite(v):
            assert f(v) == repr(v), v
    m = rng.integers(0, 5000, size=3000)
    d = rng.integers(1, 10 ** 9, size=3000)
    for a, b in zip(m, d):
        v = 2 * int(a) / int(b)                      # the reference's score, :51-52
        assert f(v) == repr(v), (a, b)


def _expected(typed, idx, cnt, score, g, stage, overall):
    gr = typed.graph
    ids = [gr.node_id(n) for n in typed.author_nodes.tolist()]
    labels = [gr.label(n) for n in typed.author_nodes.tolist()]
    out = []
    for x in range(idx.shape[0]):
        out.append("Source author global walk: {}\n".format(int(g[x])))
        for s in range(idx.shape[1]):
            y = int(idx[x, s])
            if y < 0:
                continue
            out.append("Pairwise authors walk {}: {}\n".format(ids[y], int(cnt[x, s])))
            out.append("Target author global walk: {}\n".format(int(g[y])))
            out.append("Sim score {} - {}: {}\n".format(labels[x], labels[y], float(score[x, s])))
            out.append("***Stage done in: {}\n".format(stage))
            out.append("---\n")
    if overall is not None:
        out.append("***Overall done in: {}\n".format(overall))
    return "".join(out)


@pytest.mark.parametrize("threads", [1, 3])
def test_topk_log_dblp_small_matches_python(tmp_path, dblp_small_tuples, dblp_small_expected, threads):
    from dpathsim.graph import Graph
    from dpathsim.logfmt import write_topk_log
    typed = Graph.from_tuples(*dblp_small_tuples).typed()
    e = dblp_small_expected
    idx, cnt, sc, g = e["top10_idx"].copy(), e["top10_cnt"], e["top10_score"], e["g"]
    idx[5, 7:] = -1                                   # empty slots are skipped
    path = tmp_path / "run.log"
    path.write_text("earlier run\n")
    write_topk_log(path, typed, idx, cnt, sc, g, append=True, stage_seconds=1.25e-05,
                   overall_seconds=0.5, n_threads=threads)
    want = "earlier run\n" + _expected(typed, idx, cnt, sc, g, 1.25e-05, 0.5)
    assert path.read_text(encoding="utf-8") == want


def test_topk_log_row_slice_and_overwrite(tmp_path, dblp_small_tuples, dblp_small_expected):
    from dpathsim.graph import Graph
    from dpathsim.logfmt import write_topk_log
    typed = Graph.from_tuples(*dblp_small_tuples).typed()
    e = dblp_small_expected
    r0, r1 = 100, 140
    path = tmp_path / "slice.log"
    path.write_text("stale\n")
    write_topk_log(path, typed, e["top10_idx"][r0:r1], e["top10_cnt"][r0:r1],
                   e["top10_score"][r0:r1], e["g"], row_begin=r0, append=False)
    full = _expected(typed, e["top10_idx"], e["top10_cnt"], e["top10_score"], e["g"], 0.0, None)
    blocks = full.split("Source author global walk: ")[1:]
    assert path.read_text(encoding="utf-8") == "".join(
        "Source author global walk: " + b for b in blocks[r0:r1])


def test_topk_log_rejects_bad_shapes(dblp_small_tuples):
    from dpathsim.graph import Graph
    from dpathsim.logfmt import write_topk_log
    typed = Graph.from_tuples(*dblp_small_tuples).typed()
    with pytest.raises(ValueError):
        write_topk_log("/dev/null", typed, np.zeros((2, 3), np.int32), np.zeros((2, 2), np.int64),
                       np.zeros((2, 3)), np.zeros(typed.n_authors, np.int64))
