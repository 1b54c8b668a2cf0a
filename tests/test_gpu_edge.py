"""GPU edge cases and full-size output properties (HIP path vs the oracle).

* degenerate graphs: one author (no targets: every slot empty), authors without
  papers (g = 0: 0/0 scores 0.0 and the zero-score fill), k larger than the
  number of targets (fill in reference order, then -1), no venue edges at all;
* random multigraphs with the reference's corner cases (parallel edges,
  author_of from non-author sources, papers with 0 or 2+ venues, self loops),
  for k in the one-slot-per-lane (k <= 64) and two-slot (k > 64) top-k paths;
* row slices and the dequeue order do not change any result;
* config3 at full size (all 1M rows): per-row properties that do not need the
  oracle -- scores non-increasing, ties by ascending ordinal, no self, distinct
  targets -- plus sampled (row, slot) entries re-derived bit-exactly from
  dps_pair_count and the global walks.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(v, e, k, tile_w=256):
    import pathsim_oracle as po
    from dpathsim.engine import build_engine
    from dpathsim.graph import Graph
    t = Graph.from_tuples(v, e).typed()
    if t.n_authors == 0:
        return None
    eng = build_engine(t, tile_w=tile_w)
    got = [a.cpu().numpy() for a in eng.topk(k)]
    want = po.allpairs_topk(po.OracleGraph(v, e), k)
    return got, want


def _same(got, want):
    gi, gc, gs = got
    oi, oc, os_ = want
    assert np.array_equal(gi, oi), (gi, oi)
    assert np.array_equal(gc, oc)
    assert np.array_equal(gs.view(np.int64), os_.view(np.int64))


def test_single_author_has_no_targets():
    v = [("a", "A", "author"), ("p", "P", "paper"), ("v", "V", "venue")]
    e = [("a", "p", "author_of"), ("p", "v", "submit_at")]
    got, want = _run(v, e, 5)
    _same(got, want)
    assert (got[0] == -1).all()


def test_authors_without_papers_and_large_k():
    v = [(f"a{i}", f"A{i}", "author") for i in range(6)] + \
        [("p0", "P0", "paper"), ("p1", "P1", "paper"), ("v0", "V0", "venue")]
    e = [("a0", "p0", "author_of"), ("a1", "p0", "author_of"), ("a2", "p1", "author_of"),
         ("p0", "v0", "submit_at"), ("p1", "v0", "submit_at")]
    for k in (1, 3, 5, 9):        # 5 targets per source; k = 9 leaves 4 empty slots
        got, want = _run(v, e, k)
        _same(got, want)
    assert (got[0][:, 5:] == -1).all()


def test_no_venue_edges():
    v = [(f"a{i}", f"A{i}", "author") for i in range(4)] + [("p0", "P0", "paper")]
    e = [("a0", "p0", "author_of"), ("a1", "p0", "author_of")]
    got, want = _run(v, e, 3)
    _same(got, want)
    assert (got[2] == 0.0).all()


@pytest.mark.parametrize("k", [4, 70])
def test_random_multigraphs_vs_oracle(k):
    rng = np.random.default_rng(k)
    types = ["author", "paper", "venue", "topic"]
    rels = ["author_of", "submit_at", "cites"]
    for trial in range(25):
        n = int(rng.integers(3, 90))
        ty = rng.choice(types, size=n, p=[0.45, 0.35, 0.15, 0.05])
        v = [(f"n{i}", f"L{i}", str(ty[i])) for i in range(n)]
        m = int(rng.integers(0, 6 * n))
        e = [(f"n{int(a)}", f"n{int(b)}", str(r)) for a, b, r in
             zip(rng.integers(0, n, m), rng.integers(0, n, m), rng.choice(rels, size=m))]
        res = _run(v, e, k)
        if res is not None:
            _same(*res)


def test_row_slices_and_dequeue_order_do_not_change_results():
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_dblp
    t = synth_dblp(6000, 18000, 300, seed=13).typed()
    eng = build_engine(t, tile_w=1024)
    full = [a.cpu().numpy() for a in eng.topk(10)]
    plain = [a.cpu().numpy() for a in eng.topk(10, heavy_first=False)]
    for a, b in zip(full, plain):
        assert np.array_equal(a.view(np.int64) if a.dtype == np.float64 else a,
                              b.view(np.int64) if b.dtype == np.float64 else b)
    for r0, r1 in ((0, 1), (17, 2000), (2000, 6000), (5999, 6000)):
        part = [a.cpu().numpy() for a in eng.topk(10, r0, r1)]
        for a, b in zip(part, full):
            assert np.array_equal(a, b[r0:r1])


def test_config3_full_output_properties():
    import torch
    from dpathsim import _lib
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_config
    t = synth_config("config3").typed()
    eng = build_engine(t)
    k = 10
    idx, cnt, sc = (a.cpu().numpy() for a in eng.topk(k))
    na = t.n_authors
    rows = np.arange(na)[:, None]
    assert (idx >= 0).all() and (idx < na).all()            # every author has >= k targets
    assert not (idx == rows).any()                           # self excluded
    assert (np.diff(sc, axis=1) <= 0).all()                  # scores non-increasing
    tie = np.diff(sc, axis=1) == 0
    assert (np.diff(idx, axis=1)[tie] > 0).all()             # ties by ascending ordinal
    srt = np.sort(idx, axis=1)
    assert (np.diff(srt, axis=1) > 0).all()                  # distinct targets
    assert (sc <= 1.0).all() and (cnt >= 0).all()
    # sampled entries re-derived from the pairwise walk and the global walks
    g = eng.tensor("g")[:na].cpu().numpy()
    c_ptr = eng.tensor("c_ptr")
    c_col, c_val = eng.tensor("c_col"), eng.tensor("c_val")
    out = torch.empty(1, dtype=torch.int64, device=eng.device)
    rng = np.random.default_rng(3)
    for x, s in zip(rng.integers(0, na, 300), rng.integers(0, k, 300)):
        y = int(idx[x, s])
        a0, a1, b0, b1 = (int(u) for u in c_ptr[[x, x + 1, y, y + 1]].cpu())
        _lib.call("dps_pair_count", c_col[a0:].data_ptr(), c_val[a0:].data_ptr(), a1 - a0,
                  c_col[b0:].data_ptr(), c_val[b0:].data_ptr(), b1 - b0, out.data_ptr(),
                  eng.stream)
        m = int(out.item())
        assert cnt[x, s] == m
        want = np.float64(2 * m) / np.float64(int(g[x]) + int(g[y]))
        assert sc[x, s].view(np.int64) == want.view(np.int64)


def test_topk_rows_matches_contiguous_launch():
    """dps_cct_topk_rows (arbitrary row list, repeats allowed, heaviest-first
    dequeue) gives the rows of the contiguous launch."""
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_dblp
    t = synth_dblp(6000, 18000, 300, seed=13).typed()
    eng = build_engine(t, tile_w=1024)
    full = [a.cpu().numpy() for a in eng.topk(10)]
    rng = np.random.default_rng(5)
    rows = np.concatenate([rng.integers(0, t.n_authors, 700), [0, 5999, 17, 17]])
    got = [a.cpu().numpy() for a in eng.topk_rows(10, rows)]
    for a, b in zip(got, full):
        assert np.array_equal(a.view(np.int64) if a.dtype == np.float64 else a,
                              (b.view(np.int64) if b.dtype == np.float64 else b)[rows])
    assert all(a.shape[0] == 0 for a in eng.topk_rows(10, np.zeros(0, np.int64)))


@pytest.mark.parametrize("multi,spgemm", [(1, "sort"), (3, "sort"), (3, "hash")])
def test_spgemm_long_and_huge_rows(multi, spgemm):
    """Rows of every length class, papers of 1 (single-mid path) or up to 3
    venues each (repeats dropped by the PX distinct), through the multi-mid
    SpGEMMs: expand + segmented sort/unique (the default) and the hash SpGEMM
    (lane L <= 16, LDS hash 16 < L <= 4096, global-scratch sort L > 4096) --
    C, g and the top-k against the oracle."""
    import pathsim_oracle as po
    from dpathsim.engine import build_engine
    from dpathsim.graph import Graph
    rng = np.random.default_rng(multi)
    papers_of = [5200, 1500, 40, 17, 3] + [1] * 2000
    na, nv = len(papers_of), 400
    n_pap = sum(papers_of)
    src, dst = [], []
    pid = 0
    for a, n in enumerate(papers_of):
        for _ in range(n):
            src.append(a), dst.append(na + pid)
            pid += 1
    # a few shared papers between the heavy authors and the light ones
    for _ in range(300):
        src.append(int(rng.integers(0, na))), dst.append(na + int(rng.integers(0, 6000)))
    n_ap = len(src)
    for p in range(n_pap):
        for _ in range(int(rng.integers(1, multi + 1))):
            src.append(na + p), dst.append(na + n_pap + int(rng.integers(0, nv)))
    types = np.concatenate([np.zeros(na), np.ones(n_pap), np.full(nv, 2)]).astype(np.int32)
    rel = np.concatenate([np.zeros(n_ap), np.ones(len(src) - n_ap)]).astype(np.int32)
    g = Graph(types, ["author", "paper", "venue"], np.array(src), np.array(dst), rel,
              ["author_of", "submit_at"], node_ids=lambda i: f"n{i}", labels=lambda i: f"L{i}")
    t = g.typed()
    eng = build_engine(t, tile_w=1024, spgemm=spgemm)
    co = po.COracle.from_typed(t)
    cp, cc, cv, s, gg = co.export()
    nnz = eng.info.nnz_c
    assert np.array_equal(eng.tensor("c_ptr")[: na + 1].cpu().numpy(), cp)
    assert np.array_equal(eng.tensor("c_col")[:nnz].cpu().numpy(), cc)
    assert np.array_equal(eng.tensor("c_val")[:nnz].cpu().numpy(), cv)
    assert np.array_equal(eng.tensor("s")[:nv].cpu().numpy(), s)
    assert np.array_equal(eng.tensor("g")[:na].cpu().numpy(), gg)
    _same([a.cpu().numpy() for a in eng.topk(10)], co.topk(10, 0, na))


@pytest.mark.parametrize("tile_w", [8192, 16384, 7680, 15360])
@pytest.mark.parametrize("k", [10, 100])
def test_split_rows_identical_lean(tile_w, k):
    """The lean one-wave kernel's split path (the production shape): pieces of
    the heaviest rows over several target tiles, k > 64 (two top-k registers),
    row sub-ranges -- bit for bit the unsplit rows."""
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_dblp
    t = synth_dblp(40_000, 120_000, 400, seed=17).typed()
    eng = build_engine(t, tile_w=tile_w)
    assert -(-t.n_authors // tile_w) >= 3
    whole = [a.cpu().numpy() for a in eng.topk(k, split_rows=0)]
    for r0, r1 in ((0, t.n_authors), (1000, 21000)):
        for M, P in ((256, 16), (100, 3)):
            got = [a.cpu().numpy() for a in eng.topk(k, r0, r1, split_rows=M, pieces=P)]
            for a, b in zip(got, whole):
                assert np.array_equal(a.view(np.int64) if a.dtype == np.float64 else a,
                                      (b.view(np.int64) if b.dtype == np.float64 else b)[r0:r1])


@pytest.mark.parametrize("M,P,k", [(40, 4, 10), (300, 16, 10), (64, 7, 100), (5, 64, 3)])
def test_split_rows_identical(M, P, k):
    """Heavy rows cut into target-tile pieces (dps_cct_topk_split + the merge)
    give exactly the unsplit rows, including the zero-score fill of rows with
    fewer than k positive scores and row sub-ranges."""
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_dblp
    t = synth_dblp(6000, 18000, 300, seed=13).typed()
    eng = build_engine(t, tile_w=256)
    whole = [a.cpu().numpy() for a in eng.topk(k, split_rows=0)]
    for r0, r1 in ((0, 6000), (100, 2500)):
        got = [a.cpu().numpy() for a in eng.topk(k, r0, r1, split_rows=M, pieces=P)]
        for a, b in zip(got, whole):
            assert np.array_equal(a.view(np.int64) if a.dtype == np.float64 else a,
                                  (b.view(np.int64) if b.dtype == np.float64 else b)[r0:r1])


@pytest.mark.parametrize("nv,multi", [(400, 1), (9000, 1), (9000, 3)])
def test_segment_length_classes(nv, multi):
    """Rows whose lengths sit on every boundary of the segmented sort + unique
    (lane networks <= 16 / <= 32, wave <= 64, wave LDS bitonic <= 256, block
    rank sort <= 1024, LDS bitonic <= 14336, in-place global sort above), with
    duplicate authorships (the typed CSR's distinct) and 1 or up to 3 venues
    per paper (the single-mid gather path with and without the LDS histogram,
    and the expansion path): C, s, g and the top-k against the oracle."""
    import pathsim_oracle as po
    from dpathsim.engine import build_engine
    from dpathsim.graph import Graph
    rng = np.random.default_rng(nv + multi)
    lengths = [2, 16, 17, 32, 33, 64, 65, 256, 257, 1024, 1025, 14336, 14337, 15000]
    papers_of = lengths + [1] * 300
    na = len(papers_of)
    n_pap = sum(papers_of)
    src, dst = [], []
    pid = 0
    for a, n in enumerate(papers_of):
        for _ in range(n):
            src.append(a), dst.append(na + pid)
            pid += 1
    for _ in range(500):                      # duplicate authorships
        i = int(rng.integers(0, len(src)))
        src.append(src[i]), dst.append(dst[i])
    n_ap = len(src)
    for p in range(n_pap):
        for _ in range(int(rng.integers(1, multi + 1))):
            src.append(na + p), dst.append(na + n_pap + int(rng.integers(0, nv)))
    types = np.concatenate([np.zeros(na), np.ones(n_pap), np.full(nv, 2)]).astype(np.int32)
    rel = np.concatenate([np.zeros(n_ap), np.ones(len(src) - n_ap)]).astype(np.int32)
    g = Graph(types, ["author", "paper", "venue"], np.array(src), np.array(dst), rel,
              ["author_of", "submit_at"], node_ids=lambda i: f"n{i}", labels=lambda i: f"L{i}")
    t = g.typed()
    eng = build_engine(t, tile_w=1024)
    co = po.COracle.from_typed(t)
    cp, cc, cv, s, gg = co.export()
    nnz = eng.info.nnz_c
    assert np.array_equal(eng.tensor("c_ptr")[: na + 1].cpu().numpy(), cp)
    assert np.array_equal(eng.tensor("c_col")[:nnz].cpu().numpy(), cc)
    assert np.array_equal(eng.tensor("c_val")[:nnz].cpu().numpy(), cv)
    assert np.array_equal(eng.tensor("s")[:nv].cpu().numpy(), s)
    assert np.array_equal(eng.tensor("g")[:na].cpu().numpy(), gg)
    _same([a.cpu().numpy() for a in eng.topk(10)], co.topk(10, 0, na))
