"""C-ABI boundary checks on the GPU (round 5):

* the C^T tile format decoded exactly as include/dpathsim.h documents it
  (tile_w 8192 / 16384 / 32768) re-sums to the oracle's C, bucket by bucket;
* dps_ct_tiles_build2 with an undersized nnz_cap reports DPS_ERR_OVERFLOW;
* dps_ct_tiles_sums against host sums of the same buckets;
* the optimistic 4-bit passes (engine.opt_passes, the OPT instantiation of
  k_cct1) against the oracle, with and without venue skipping, and on a
  crafted graph where counts of 16 and more overflow the nibbles;
* dps_unpack_gathered never writes past n_rows when the device edges describe
  more rows.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cmp(got, want):
    gi, gc, gs = (a.cpu().numpy() for a in got)
    oi, oc, os_ = want
    bad = np.flatnonzero((gi != oi).any(1) | (gc != oc).any(1) |
                         (gs.view(np.int64) != os_.view(np.int64)).any(1))
    assert len(bad) == 0, (f"{len(bad)} rows differ; first row {bad[0]}:\n"
                           f"gpu {gi[bad[0]]} {gc[bad[0]]} {gs[bad[0]]}\n"
                           f"orc {oi[bad[0]]} {oc[bad[0]]} {os_[bad[0]]}")


def decode_tiles(off, ent, n_mids, n_targets, tile_w):
    """Decode tile_off / tile_ent per include/dpathsim.h (dps_ct_tiles_build):
    returns (v, label, value) arrays of every non-padding piece and checks the
    16-byte padding of every bucket."""
    T = -(-n_targets // tile_w)
    off = off[: n_mids * T + 1].astype(np.int64)
    nw = np.diff(off)
    assert (nw % 4 == 0).all(), "a bucket is not padded to 16 bytes"
    b_of_word = np.repeat(np.arange(n_mids * T), nw)
    words = ent[: off[-1]].astype(np.uint32)
    if tile_w >= 32768:                      # uint32 (C << 16) | l, C = 0 padding
        c = (words >> 16).astype(np.int64)
        l = (words & 0xFFFF).astype(np.int64)
        keep = c > 0
        b = b_of_word[keep]
        return b // T, (b % T) * tile_w + l[keep], c[keep]
    h = words.view(np.uint16).astype(np.int64)          # two per word, low half first
    b = np.repeat(b_of_word, 2)
    if tile_w <= 8192:                       # (l << 3) | e; e = 6, 7 at l % 4 == 3 pad
        l, e = h >> 3, h & 7
        pad = ((l & 3) == 3) & (e >= 6)
    else:                                    # 16384 / 15360: (l << 2) | e; e = 2, 3 at l % 8 == 7 pad
        l, e = h >> 2, h & 3
        pad = ((l & 7) == 7) & (e >= 2)
    keep = ~pad
    b = b[keep]
    return b // T, (b % T) * tile_w + l[keep], np.left_shift(1, e[keep])


@pytest.mark.parametrize("tile_w", [8192, 16384, 32768, 7680, 15360])
def test_tile_format_decodes_to_c(tile_w):
    """Every C^T bucket decoded per the header sums to C[y, v] of the oracle
    (y = t_perm[label]), tile_maxc is the bucket maximum, tile_gmin the tile's
    smallest g; and the same for the companion u8 tiles at 16384."""
    import pathsim_oracle as po
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_config
    t = synth_config("config3", scale=0.05).typed()
    eng = build_engine(t, tile_w=tile_w)
    NA, NV = t.n_authors, t.n_mids
    cp, cc, cv, s, g = po.COracle.from_typed(t).export()
    row = np.repeat(np.arange(NA), np.diff(cp))
    want = np.zeros((NA, NV), np.int64)
    want[row, cc[: cp[-1]]] = cv[: cp[-1]]
    perm = eng.tensor("t_perm")[:NA].cpu().numpy().astype(np.int64)
    sets = [(tile_w, "tile_off", "tile_ent", "tile_maxc")]
    if tile_w in (16384, 15360):
        sets.append((tile_w // 2, "half_off", "half_ent", "half_maxc"))
    for w, o_n, e_n, m_n in sets:
        off = eng.tensor(o_n).cpu().numpy().view(np.uint32)
        ent = eng.tensor(e_n).cpu().numpy().view(np.uint32)
        v, lab, val = decode_tiles(off, ent, NV, NA, w)
        assert (lab < NA).all()
        got = np.zeros((NA, NV), np.int64)
        np.add.at(got, (perm[lab], v), val)
        assert np.array_equal(got, want), f"decoded C differs at tile_w {w}"
        T = -(-NA // w)
        mx = np.zeros(NV * T, np.int64)
        yl = np.argsort(perm)               # label of every target
        b = cc[: cp[-1]].astype(np.int64) * T + yl[row] // w
        np.maximum.at(mx, b, cv[: cp[-1]].astype(np.int64))
        gm = eng.tensor(m_n)[: NV * T].cpu().numpy().astype(np.int64)
        assert np.array_equal(gm, mx), f"tile_maxc differs at tile_w {w}"
    T = -(-NA // tile_w)
    gmin = np.array([g[perm[i * tile_w:(i + 1) * tile_w]].min() for i in range(T)])
    assert np.array_equal(eng.tensor("tile_gmin")[:T].cpu().numpy(), gmin)


def test_tiles_build2_undersized_cap_reports_overflow(tune):
    """dps_ct_tiles_build2 (sorted layout) with nnz_cap below nnz(C): the device
    reports DPS_ERR_OVERFLOW, and the exact cap builds the same tiles as the
    engine with status 0."""
    from dpathsim import _lib
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_dblp
    tune(_lib.TUNE_TILE_BUILD, 2)
    t = synth_dblp(6_000, 24_000, 20_000, seed=31).typed()
    tile_w = 8192
    eng = build_engine(t, tile_w=tile_w)
    d = eng._dev
    NA, NV = t.n_authors, t.n_mids
    nnz = int(d["c_ptr"][NA].item())
    T = -(-NA // tile_w)
    for cap, want in ((nnz, 0), (nnz - 1, _lib.DPS_ERR_OVERFLOW), (nnz // 2, _lib.DPS_ERR_OVERFLOW)):
        off = torch.empty(NV * T + 1, dtype=torch.int32, device=eng.device)
        ent = torch.zeros_like(d["tile_ent"])
        st = torch.full((1,), 7, dtype=torch.int32, device=eng.device)
        ws = torch.empty(_lib.size("dps_ct_tiles_workspace_size2", NV, NA, tile_w, cap),
                         dtype=torch.uint8, device=eng.device)
        _lib.call("dps_ct_tiles_build2", d["c_ptr"].data_ptr(), d["c_col"].data_ptr(),
                  d["c_val"].data_ptr(), None, d["t_rank"].data_ptr(), NA, NV, tile_w, cap,
                  off.data_ptr(), ent.data_ptr(), None, None, st.data_ptr(), ws.data_ptr(),
                  ws.numel(), eng.stream)
        torch.cuda.synchronize()
        assert int(st.item()) == want, (cap, nnz, int(st.item()))
        if want == 0:
            assert torch.equal(off, d["tile_off"][: NV * T + 1])


@pytest.mark.parametrize("w", [8192, 16384])
def test_tiles_sums_match_host(w):
    """dps_ct_tiles_sums = the sum of the decoded pieces of each bucket."""
    from dpathsim import _lib
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_config
    t = synth_config("config3", scale=0.05).typed()
    eng = build_engine(t, tile_w=w)
    NA, NV = t.n_authors, t.n_mids
    T = -(-NA // w)
    off_t, ent_t = eng.tensor("tile_off"), eng.tensor("tile_ent")
    out = torch.empty(NV * T, dtype=torch.int32, device=eng.device)
    _lib.call("dps_ct_tiles_sums", off_t.data_ptr(), ent_t.data_ptr(), NV * T, w, out.data_ptr(),
              eng.stream)
    torch.cuda.synchronize()
    v, lab, val = decode_tiles(off_t.cpu().numpy().view(np.uint32),
                               ent_t.cpu().numpy().view(np.uint32), NV, NA, w)
    want = np.bincount(v * T + lab // w, weights=val, minlength=NV * T).astype(np.int64)
    assert np.array_equal(out.cpu().numpy().astype(np.int64), want)


def _clique_graph(n_fill=40_000, seed=3):
    """Groups of authors who each publish at the same 18-24 venues (one or two
    papers per venue): their pairwise counts are 18..96 while their tile bounds
    stay within 255, so the optimistic 4-bit passes run on them and overflow;
    filler authors spread the targets over three 16384-target tiles."""
    from dpathsim.graph import Graph
    rng = np.random.default_rng(seed)
    nv = 300
    src, dst = [], []
    pid = 0
    na = 0
    venue = []
    groups = []
    for gi in range(12):
        size = int(rng.integers(20, 60))
        vs = rng.choice(nv, int(rng.integers(18, 25)), replace=False)
        groups.append((na, size, vs))
        na += size
    n_grp = na
    na += n_fill
    for a0, size, vs in groups:
        for a in range(a0, a0 + size):
            for v in vs:
                for _ in range(1 + int(rng.random() < 0.3)):
                    src.append(a)
                    dst.append(pid)
                    venue.append(v)
                    pid += 1
    for i in range(n_fill):                     # filler: 1-3 papers at random venues
        for _ in range(int(rng.integers(1, 4))):
            src.append(n_grp + i)
            dst.append(pid)
            venue.append(int(rng.integers(0, nv)))
            pid += 1
    n_pap = pid
    src = np.array(src) ; dst = np.array(dst) + na
    venue = np.array(venue)
    src = np.concatenate([src, na + np.arange(n_pap)])
    dst = np.concatenate([dst, na + n_pap + venue])
    types = np.concatenate([np.zeros(na), np.ones(n_pap), np.full(nv, 2)]).astype(np.int32)
    rel = np.concatenate([np.zeros(len(src) - n_pap), np.ones(n_pap)]).astype(np.int32)
    perm = rng.permutation(na)                   # groups spread over the tiles
    inv = np.empty(na, np.int64)
    inv[perm] = np.arange(na)
    is_a = src < na
    src = np.where(is_a, inv[np.minimum(src, na - 1)], src)
    return Graph(types, ["author", "paper", "venue"], src, dst, rel, ["author_of", "submit_at"],
                 node_ids=lambda i: f"n{i}", labels=lambda i: f"L{i}")


@pytest.mark.parametrize("vs", [True, False])
@pytest.mark.parametrize("case", ["config3_20", "cliques"])
def test_opt_passes_exact(case, vs):
    import pathsim_oracle as po
    from dpathsim.engine import build_engine
    from dpathsim.synth import synth_config
    if case == "config3_20":
        t = synth_config("config3", scale=0.05).typed()
    else:
        t = _clique_graph().typed()
    eng = build_engine(t, tile_w=16384, venue_skip=vs)
    co = po.COracle.from_typed(t)
    want = co.topk(10, 0, t.n_authors)
    eng.opt_passes = True
    eng.build()
    assert eng.tensor("tile_sum") is not None
    got = eng.topk(10, heavy_first=False)     # one plain launch: the counters are its own
    torch.cuda.synchronize()
    kc = eng.kernel_counts()
    _cmp(got, want)
    if case == "cliques":
        assert kc["opt_redo"] > 0, kc            # the overflow check fired and the redo ran
        assert want[1].max() >= 16
    _cmp(eng.topk(10), want)                     # bench path: heavy-first, split, merge


def test_unpack_gathered_clamps_to_n_rows():
    """Device edges spanning more rows than n_rows: only n_rows rows written."""
    from dpathsim import _lib
    k, m, world = 4, 5, 2
    dev = "cuda"
    edges = torch.tensor([0, 5, 10], dtype=torch.int64, device=dev)
    words = torch.arange(world * m * k, dtype=torch.int64, device=dev) % 7
    words = (words << 32) | (torch.arange(world * m * k, device=dev) % 9)
    den = torch.ones(16, dtype=torch.int64, device=dev)
    n_rows = 6                                   # < edges[world] - edges[0] = 10
    oi = torch.full((n_rows + 4, k), -5, dtype=torch.int32, device=dev)
    oc = torch.full((n_rows + 4, k), -5, dtype=torch.int64, device=dev)
    os_ = torch.full((n_rows + 4, k), -5.0, dtype=torch.float64, device=dev)
    _lib.call("dps_unpack_gathered", words.data_ptr(), world, m, k, edges.data_ptr(), n_rows,
              den.data_ptr(), oi.data_ptr(), oc.data_ptr(), os_.data_ptr(),
              torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert (oi[n_rows:] == -5).all() and (oc[n_rows:] == -5).all()
    w = words.cpu().numpy().reshape(world * m, k)
    want_i = (w[:n_rows] & 0xFFFFFFFF).astype(np.int32)
    assert np.array_equal(oi[:n_rows].cpu().numpy(), want_i)
