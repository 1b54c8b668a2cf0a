"""The N > 1 build's tile split on one GPU:
every rank builds the C^T tiles of its own target-tile range from the sub-C
of its labels (dps_label_rows + dps_ct_tiles_build2), packs them into a slice
(dps_tiles_pack), the slices are all-gathered, and dps_tiles_assemble rebuilds
the full layout.  Here the ranks run one after the other in one process (the
all-gather is a copy), so any world size can be checked on one GPU: the
assembled offsets, maxima and tile minima equal the single-GPU build's, every
bucket holds the same entries, and the hot kernel over the assembled tiles
gives the oracle's top-k bit for bit."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


class _Recorder:
    """A TileSplit stand-in for rank r of `world`: its all-gather keeps the
    slice it is sent (calls in build order) and hands back `slices` where
    provided; its max over ranks records the values it is sent and returns
    `maxima` (in call order) where provided."""

    def __init__(self, rank, world, slices=None, maxima=None):
        self.rank, self.world = rank, world
        self.sent, self.slices = [], slices
        self.caps = {}
        self.calls = 0
        self.seen, self.maxima = [], maxima

    def allgather(self, send, recv):
        self.sent.append(send.clone())
        if self.slices is not None:
            recv.copy_(torch.cat([s[self.calls] for s in self.slices]))
        else:                          # recording: an empty (all-zero) gather
            recv.zero_()
        self.calls += 1

    def allreduce_max(self, v):
        self.seen.append(int(v))
        return int(self.maxima[len(self.seen) - 1]) if self.maxima else int(v)


def _bucket_multisets_equal(off_a, ent_a, off_b, ent_b, w):
    """Every bucket holds the same real entries (16-bit pieces; the padding
    codes of include/dpathsim.h, whose labels only spread the no-op adds over
    the banks, are left out: they depend on the bucket's index in its build)."""
    n = int(off_a[-1]) * 2
    a, b = ent_a.view(np.uint16)[:n].astype(np.int64), ent_b.view(np.uint16)[:n].astype(np.int64)
    bucket = np.repeat(np.arange(len(off_a) - 1), 2 * np.diff(off_a))

    def real(h):
        if w <= 8192:
            return ~((((h >> 3) & 3) == 3) & ((h & 7) >= 6))
        return ~((((h >> 2) & 7) == 7) & ((h & 3) >= 2))
    ka, kb = real(a), real(b)
    a, ba, b, bb = a[ka], bucket[ka], b[kb], bucket[kb]
    return len(a) == len(b) and np.array_equal(a[np.lexsort((a, ba))], b[np.lexsort((b, bb))])


def _record(t, world, tile_w, maxima):
    out = []
    for r in range(world):
        e = PathSimEngine_(t, tile_w=tile_w)
        e.split = _Recorder(r, world, maxima=maxima)
        e.upload().build(check=False)
        torch.cuda.synchronize()
        out.append(e.split)
        del e
    return out


def PathSimEngine_(*a, **kw):
    from dpathsim.engine import PathSimEngine
    return PathSimEngine(*a, **kw)


def _split_engine(t, world, tile_w=None):
    """Every rank's first build: the plan (each rank's real slice size, one
    max per tile width); then every rank's slices at the plan's capacity
    (recorded), and rank 0's engine with the gathered slices."""
    seen = [s.seen for s in _record(t, world, tile_w, None)]
    maxima = [max(v[i] for v in seen) for i in range(len(seen[0]))]
    recs = [s.sent for s in _record(t, world, tile_w, maxima)]
    eng = PathSimEngine_(t, tile_w=tile_w)
    eng.split = _Recorder(0, world, slices=recs, maxima=maxima)
    eng.upload().build()
    return eng


@pytest.mark.parametrize("world", [2, 3, 8])
def test_split_tiles_equal_single_gpu_build(world):
    import pathsim_oracle as po
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_config
    t = synth_config("config3", scale=0.05).typed()      # 4 tiles of 16384, 7 of 8192
    ref = build_engine(t)
    eng = _split_engine(t, world)
    NA, NV = t.n_authors, t.n_mids
    for w, o_n, e_n, m_n in ((16384, "tile_off", "tile_ent", "tile_maxc"),
                             (8192, "half_off", "half_ent", "half_maxc")):
        T = -(-NA // w)
        oa = ref.tensor(o_n)[: NV * T + 1].cpu().numpy().view(np.uint32).astype(np.int64)
        ob = eng.tensor(o_n)[: NV * T + 1].cpu().numpy().view(np.uint32).astype(np.int64)
        assert np.array_equal(oa, ob), f"offsets differ at {w}"
        assert torch.equal(ref.tensor(m_n)[: NV * T], eng.tensor(m_n)[: NV * T]), w
        assert _bucket_multisets_equal(oa, ref.tensor(e_n).cpu().numpy(), ob,
                                       eng.tensor(e_n).cpu().numpy(), w), f"entries differ at {w}"
    T = -(-NA // 16384)
    assert torch.equal(ref.tensor("tile_gmin")[:T], eng.tensor("tile_gmin")[:T])
    want = po.COracle.from_typed(t).topk(10, 0, NA)
    got = [a.cpu().numpy() for a in eng.topk(10)]
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
    assert np.array_equal(got[2].view(np.int64), want[2].view(np.int64))


@pytest.mark.parametrize("tile_w", [8192, 32768])
def test_split_tiles_other_widths_and_many_mids(tile_w, tune):
    """u8 (8192) and 32-bit (32768) tiles, and 20k mids (the sorted build)."""
    import pathsim_oracle as po
    from dpathsim import _lib
    from dpathsim.synth import synth_dblp
    tune(_lib.TUNE_TILE_BUILD, 2)
    t = synth_dblp(70_000, 200_000, 20_000, seed=31).typed()
    eng = _split_engine(t, 3, tile_w=tile_w)
    want = po.COracle.from_typed(t).topk(10, 0, t.n_authors)
    got = [a.cpu().numpy() for a in eng.topk(10)]
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
    assert np.array_equal(got[2].view(np.int64), want[2].view(np.int64))


def test_split_slice_overflow_is_reported():
    """A gather capacity below a slice's entries: dps_tiles_pack flags it and
    check() raises instead of using a truncated layout."""
    from dpathsim.engine import PathSimEngine
    from dpathsim.synth import synth_config
    t = synth_config("config3", scale=0.05).typed()
    recs = []
    for r in range(2):
        e = PathSimEngine(t)
        e.split = _Recorder(r, 2, maxima=[64, 64])
        e.upload().build(check=False)
        recs.append(e.split.sent)
    eng = PathSimEngine(t)
    eng.split = _Recorder(0, 2, slices=recs, maxima=[64, 64])
    with pytest.raises(RuntimeError, match="gather capacity"):
        eng.upload().build()


def test_split_plan_is_per_graph():
    """one TileSplit reused for a second, larger graph must not
    gather with the first graph's capacity (the plan is keyed by the graph);
    the second graph's assembled tiles still give the oracle's top-k."""
    import pathsim_oracle as po
    from dpathsim.synth import synth_config
    small = synth_config("config3", scale=0.01).typed()
    big = synth_config("config3", scale=0.05).typed()
    # world 2, one split object for both graphs: two plans, the slices of
    # each graph at its own capacity
    maxima_small = [max(v[i] for v in (s.seen for s in _record(small, 2, None, None)))
                    for i in range(2)]
    maxima_big = [max(v[i] for v in (s.seen for s in _record(big, 2, None, None)))
                  for i in range(2)]
    assert maxima_big[0] > maxima_small[0]
    recs_small = [s.sent for s in _record(small, 2, None, maxima_small)]
    recs_big = [s.sent for s in _record(big, 2, None, maxima_big)]
    shared = _Recorder(0, 2, slices=recs_small, maxima=maxima_small + maxima_big)
    e1 = PathSimEngine_(small)
    e1.split = shared
    e1.upload().build()
    shared.slices, shared.calls = recs_big, 0
    e2 = PathSimEngine_(big)
    e2.split = shared
    e2.upload().build()
    assert len(shared.caps) == 4 and len(shared.seen) == 4
    want = po.COracle.from_typed(big).topk(10, 0, big.n_authors)
    got = [a.cpu().numpy() for a in e2.topk(10)]
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
    assert np.array_equal(got[2].view(np.int64), want[2].view(np.int64))


@pytest.mark.parametrize("tile_w", [16384, 15360])
def test_dual_build_equals_two_builds(tile_w):
    """dps_ct_tiles_build_dual (round 6: both tile sets and the heavy-venue
    table from one walk of C) against two dps_ct_tiles_build2 calls and
    dps_heavy_table: offsets, maxima, tile minima and the heavy table bit for
    bit, every bucket's entries as a multiset."""
    from dpathsim.engine import PathSimEngine
    from dpathsim.synth import synth_config
    t = synth_config("config3", scale=0.05).typed()
    engs = []
    for dual in (True, False):
        e = PathSimEngine(t, tile_w=tile_w)
        e.dual_build = dual
        e.upload().build()
        engs.append(e)
    a, b = engs
    NA, NV = t.n_authors, t.n_mids
    for w, o_n, e_n, m_n in ((tile_w, "tile_off", "tile_ent", "tile_maxc"),
                             (tile_w // 2, "half_off", "half_ent", "half_maxc")):
        T = -(-NA // w)
        oa = a.tensor(o_n)[: NV * T + 1].cpu().numpy().view(np.uint32).astype(np.int64)
        ob = b.tensor(o_n)[: NV * T + 1].cpu().numpy().view(np.uint32).astype(np.int64)
        assert np.array_equal(oa, ob), f"offsets differ at {w}"
        assert torch.equal(a.tensor(m_n)[: NV * T], b.tensor(m_n)[: NV * T]), w
        assert _bucket_multisets_equal(oa, a.tensor(e_n).cpu().numpy(), ob,
                                       b.tensor(e_n).cpu().numpy(), w), f"entries differ at {w}"
    T = -(-NA // tile_w)
    assert torch.equal(a.tensor("tile_gmin")[:T], b.tensor("tile_gmin")[:T])
    assert a.tensor("hv_c") is not None and torch.equal(a.tensor("hv_c"), b.tensor("hv_c"))
    assert torch.equal(a.tensor("hv_slot"), b.tensor("hv_slot"))
