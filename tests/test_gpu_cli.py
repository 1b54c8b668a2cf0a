"""GPU: the command line (``python -m dpathsim``) and the ``diag`` denominator.

* ``--source-name``: the reference's single-source run() (DPathSim_APVPA.py:
  28-68) on a GEXF the CLI reads itself -- log equal to the oracle's lines;
* ``--all-pairs``: the native log writer's blocks equal the oracle's top-k
  rendered in the reference's format, for both denominators;
* ``diag``: the hot kernel with M[x,x] + M[y,y] against the oracle variant.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _gexf(tmp_path, dblp_small_tuples):
    from dpathsim.gexf import write_gexf
    from dpathsim.graph import Graph
    p = tmp_path / "dblp_small.gexf"
    write_gexf(Graph.from_tuples(*dblp_small_tuples), str(p))
    return str(p)


def _no_timing(lines):
    return [ln for ln in lines if not ln.startswith("***")]


def test_cli_single_source(tmp_path, dblp_small_tuples):
    import pathsim_oracle as po
    from dpathsim.cli import main
    v, e = dblp_small_tuples
    path = _gexf(tmp_path, dblp_small_tuples)
    og = po.OracleGraph(v, e)
    src = og.authors[17]
    log = tmp_path / "single.log"
    assert main(["--graph", path, "--source-name", og.labels[src], "--out", str(log),
                 "--quiet"]) == 0
    got = [ln for ln in log.read_text().splitlines() if ln != "---"]
    assert _no_timing(got) == po.single_source_log_lines(og, src)


@pytest.mark.parametrize("den", ["rowsum", "diag"])
def test_cli_all_pairs_log(tmp_path, dblp_small_tuples, den):
    import pathsim_oracle as po
    from dpathsim.cli import main
    v, e = dblp_small_tuples
    path = _gexf(tmp_path, dblp_small_tuples)
    log = tmp_path / f"all_{den}.log"
    k = 5
    assert main(["--graph", path, "--all-pairs", "--topk", str(k), "--denominator", den,
                 "--out", str(log)]) == 0
    og = po.OracleGraph(v, e)
    idx, cnt, sc = po.allpairs_topk(og, k, denominator=den)
    d = og.g        # the walk lines print the global walk under either denominator
    want = []
    for x, a in enumerate(og.authors):
        want.append(f"Source author global walk: {int(d[x])}")
        for s in range(k):
            y = int(idx[x, s])
            if y < 0:
                continue
            b = og.authors[y]
            want += [f"Pairwise authors walk {b}: {int(cnt[x, s])}",
                     f"Target author global walk: {int(d[y])}",
                     f"Sim score {og.labels[a]} - {og.labels[b]}: {float(sc[x, s])}", "---"]
    assert _no_timing(log.read_text().splitlines()) == want


@pytest.mark.parametrize("tile_w", [512, 8192, 16384])
def test_diag_denominator_vs_oracle(tile_w):
    import pathsim_oracle as po
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_dblp
    t = synth_dblp(20_000, 60_000, 500, seed=7).typed()
    eng = build_engine(t, tile_w=tile_w, denominator="diag")
    co = po.COracle.from_typed(t)
    assert np.array_equal(eng.tensor("diag")[: t.n_authors].cpu().numpy(), co.diag())
    gi, gc, gs = (a.cpu().numpy() for a in eng.topk(10))
    oi, oc, os_ = co.topk_rows(10, np.arange(t.n_authors), denominator="diag")
    assert np.array_equal(gi, oi) and np.array_equal(gc, oc)
    assert np.array_equal(gs.view(np.int64), os_.view(np.int64))
