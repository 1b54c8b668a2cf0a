"""Multi-rank row sharding + top-k gather (dpathsim.dist) on CPU with gloo.

The GPU path runs the same code with the nccl (RCCL) backend in bench.py.  The
CPU tests here take each shard's top-k from the C oracle; the ``gpu``-marked
test at the end computes the shards with the HIP engine (two gloo ranks on one
GPU) and checks the gathered result against the oracle.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dpathsim.dist import (balanced_bounds, gather_topk, gather_topk_compact, max_shard,
                           pack_topk, read_topk_shards, shard_bounds, unpack_topk,
                           write_topk_shard)


@pytest.mark.parametrize("n", [0, 1, 7, 1000, 1_000_003])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shards_partition_rows(n, world):
    bounds = [shard_bounds(n, r, world) for r in range(world)]
    assert bounds[0][0] == 0 and bounds[-1][1] == n
    for (a, b), (c, _) in zip(bounds, bounds[1:]):
        assert b == c and a <= b
    sizes = [b - a for a, b in bounds]
    assert max(sizes) - min(sizes) <= 1
    assert max_shard(n, world) == max(sizes)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_balanced_bounds_partition_and_balance(world):
    rng = np.random.default_rng(world)
    w = torch.from_numpy(rng.pareto(1.2, 100_000).astype(np.int64) + 1)
    b = balanced_bounds(w, world)
    assert b[0][0] == 0 and b[-1][1] == len(w)
    assert all(x[1] == y[0] for x, y in zip(b, b[1:]))
    loads = [int(w[a:c].sum()) for a, c in b]
    assert max(loads) - min(loads) <= 2 * int(w.max())    # balanced up to one row per cut
    assert balanced_bounds(torch.zeros(0, dtype=torch.int64), world) == [(0, 0)] * world


@pytest.mark.parametrize("world", [1, 2, 5, 8])
def test_balanced_edges_match_bounds(world):
    """bench.py re-derives the shards inside the timed step as a tensor
    (balanced_edges, nothing read back); it must equal the host bounds."""
    from dpathsim.dist import balanced_edges
    rng = np.random.default_rng(3 + world)
    w = torch.from_numpy(rng.pareto(1.1, 50_000).astype(np.int64) + 1)
    e = balanced_edges(w, world).tolist()
    b = balanced_bounds(w, world)
    assert [(e[r], e[r + 1]) for r in range(world)] == b
    assert balanced_edges(torch.zeros(0, dtype=torch.int64), world).tolist() == [0] * (world + 1)


def _worker(rank, world, port, k, result_path, balanced=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import pathsim_oracle as po
        from dpathsim.synth import synth_dblp
        t = synth_dblp(1500, 4500, 120, seed=21).typed()
        co = po.COracle.from_typed(t)
        na = t.n_authors
        bounds = None
        if balanced:      # shards by per-row work sum_{v in x} n_v (as PathSimEngine.row_work)
            cp, cc = co.export()[:2]
            n_v = np.bincount(cc, minlength=t.n_mids)
            pre = np.concatenate([[0], np.cumsum(n_v[cc])])
            bounds = balanced_bounds(torch.from_numpy(pre[cp[1:]] - pre[cp[:-1]]), world)
        r0, r1 = bounds[rank] if bounds else shard_bounds(na, rank, world)
        m = max_shard(na, world, bounds)
        oi, oc, os_ = co.topk(k, r0, r1, threads=1)
        parts = []
        for a, dt in ((oi, torch.int32), (oc, torch.int64), (os_, torch.float64)):
            p = torch.zeros((m, k), dtype=dt)
            p[: r1 - r0] = torch.from_numpy(a)
            parts.append(p)
        res = gather_topk(tuple(parts), na, world, bounds=bounds)
        # the 8-byte wire format: counts and indices only, scores rebuilt on rank 0
        g = torch.from_numpy(co.export()[4][:na].astype(np.int64))
        res8 = gather_topk_compact(tuple(parts[:2]), g, na, world, bounds=bounds)
        shard_dir = result_path + ".shards"
        write_topk_shard(shard_dir, rank, world, bounds or [shard_bounds(na, r, world)
                                                           for r in range(world)], tuple(parts), k)
        dist.barrier()
        if rank != 0:
            assert res is None and res8 is None   # gathered to rank 0 only
        else:
            fi, fc, fs = co.topk(k, 0, na, threads=1)
            ok = True
            for gi, gc, gs in (res, res8, read_topk_shards(shard_dir)):
                ok = ok and (np.array_equal(gi.numpy(), fi) and np.array_equal(gc.numpy(), fc)
                             and np.array_equal(gs.numpy().view(np.int64), fs.view(np.int64)))
            with open(result_path, "w") as f:
                f.write("ok" if ok else "mismatch")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("balanced", [False, True])
@pytest.mark.parametrize("world", [2, 3])
def test_gloo_gather_equals_single_rank(tmp_path, world, balanced):
    out = tmp_path / "result.txt"
    mp.start_processes(_worker, args=(world, _free_port(), 10, str(out), balanced), nprocs=world,
                       join=True, start_method="spawn")
    assert out.read_text() == "ok"


def test_compact_rescore_matches_kernel_division():
    """rescore() rebuilds score = double(2 cnt) / double(den[x] + den[y]) bit for
    bit (the oracle's scores), 0.0 for zero counts and -1 slots."""
    import pathsim_oracle as po
    from dpathsim.dist import pack_counts, rescore
    from dpathsim.synth import synth_dblp
    t = synth_dblp(3000, 9000, 150, seed=4).typed()
    co = po.COracle.from_typed(t)
    g = torch.from_numpy(co.export()[4][: t.n_authors].astype(np.int64))
    oi, oc, os_ = co.topk(10, 100, 700, threads=1)
    oi[5, 9], oc[5, 9], os_[5, 9] = -1, 0, 0.0            # an empty slot
    i2, c2, s2 = rescore(pack_counts(torch.from_numpy(oi), torch.from_numpy(oc)), g, 100)
    assert np.array_equal(i2.numpy(), oi) and np.array_equal(c2.numpy(), oc)
    assert np.array_equal(s2.numpy().view(np.int64), os_.view(np.int64))


@pytest.mark.parametrize("world", [1, 2, 5, 8])
def test_shard_edges_host_equals_row_work_plan(world):
    """shard_edges(terms) (bench.py's plan over the build's row work terms)
    equals balanced_edges over PathSimEngine.row_work() = terms + half the mean."""
    from dpathsim.dist import balanced_edges, shard_edges
    rng = np.random.default_rng(11 + world)
    terms = torch.from_numpy(rng.pareto(1.1, 40_000).astype(np.int64) * 100)
    work = terms + (terms.sum() // terms.numel()) // 2
    assert shard_edges(terms, world).tolist() == balanced_edges(work, world).tolist()
    ref = shard_edges(terms, world)
    mism = torch.zeros(1, dtype=torch.int64)
    shard_edges(terms, world, ref=ref, mismatch=mism)
    assert int(mism) == 0
    pert = terms + 7 * (torch.arange(terms.numel()) % 3 == 0)
    want = int((shard_edges(pert, world) != ref).sum())
    shard_edges(pert, world, ref=ref, mismatch=mism)
    assert int(mism) == want
    if world > 1:                       # a reference plan off by one edge: exactly one mismatch
        bad = ref.clone()
        bad[1] += 1
        mism.zero_()
        shard_edges(terms, world, ref=bad, mismatch=mism)
        assert int(mism) == 1
    assert shard_edges(torch.zeros(0, dtype=torch.int64), world).tolist() == [0] * (world + 1)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2, 3, 8, 255])
def test_shard_edges_device_equals_host(world):
    """dps_shard_edges (HIP) gives the host plan's edges bit for bit and counts
    the edges that differ from a reference plan."""
    from dpathsim.dist import shard_edges
    rng = np.random.default_rng(world)
    for n in (1, 7, 1000, 300_001):
        terms = torch.from_numpy(rng.pareto(1.2, n).astype(np.int64) * 50)
        host = shard_edges(terms, world)
        dev = shard_edges(terms.cuda(), world)
        assert dev.cpu().tolist() == host.tolist(), n
        mism = torch.zeros(1, dtype=torch.int64, device="cuda")
        shard_edges(terms.cuda(), world, ref=dev, mismatch=mism)
        assert int(mism.item()) == 0
        bad = dev.clone()
        if world > 1:
            bad[1] += 1
            shard_edges(terms.cuda(), world, ref=bad, mismatch=mism)
            assert int(mism.item()) == 1
    z = shard_edges(torch.zeros(0, dtype=torch.int64, device="cuda"), world)
    assert z.cpu().tolist() == [0] * (world + 1)


@pytest.mark.gpu
def test_pack_unpack_gathered_device():
    """dps_pack_counts / dps_unpack_gathered (HIP) against the host PyTorch
    words and rescore: shards of unequal size in a [world * m, k] buffer, -1
    slots and zero counts, rows in order, scores bit for bit."""
    from dpathsim.dist import pack_counts, rescore, unpack_gathered
    rng = np.random.default_rng(5)
    na, k, world = 5000, 7, 3
    den = torch.from_numpy(rng.integers(1, 10 ** 9, na).astype(np.int64))
    idx = torch.from_numpy(rng.integers(-1, na, (na, k)).astype(np.int32))
    cnt = torch.from_numpy(rng.integers(0, 2 ** 31 - 1, (na, k)).astype(np.int64))
    cnt[idx < 0] = 0
    cnt[::11, 0] = 0
    host_words = pack_counts(idx, cnt)
    dev_words = pack_counts(idx.cuda(), cnt.cuda())
    assert torch.equal(dev_words.cpu(), host_words)
    edges = [0, 1200, 1200 + 2100, na]                  # shard sizes 1200, 2100, 1700
    m = 2100
    g = torch.full((world * m, k), -12345, dtype=torch.int64)
    for r in range(world):
        g[r * m: r * m + edges[r + 1] - edges[r]] = host_words[edges[r]:edges[r + 1]]
    ei = torch.tensor(edges, dtype=torch.int64, device="cuda")
    di, dc, ds = unpack_gathered(g.cuda(), world, m, ei, den.cuda())
    hi, hc, hs = rescore(host_words, den, 0)
    assert torch.equal(di.cpu(), hi) and torch.equal(dc.cpu(), hc)
    assert torch.equal(ds.cpu().view(torch.int64), hs.view(torch.int64))
    # a row range that does not start at 0 (a rank's slice, world 1)
    si, sc_, ss = rescore(dev_words[300:900], den.cuda(), 300)
    hi, hc, hs = rescore(host_words[300:900], den, 300)
    assert torch.equal(si.cpu(), hi) and torch.equal(ss.cpu().view(torch.int64), hs.view(torch.int64))


def test_pack_roundtrip():
    rng = np.random.default_rng(0)
    idx = torch.from_numpy(rng.integers(-1, 2 ** 31 - 1, (50, 7)).astype(np.int32))
    cnt = torch.from_numpy(rng.integers(0, 2 ** 31 - 1, (50, 7)).astype(np.int64))
    sc = torch.from_numpy(rng.random((50, 7)))
    sc[0, 0] = 0.0
    i2, c2, s2 = unpack_topk(pack_topk(idx, cnt, sc))
    assert torch.equal(i2, idx) and torch.equal(c2, cnt)
    assert torch.equal(s2.view(torch.int64), sc.view(torch.int64))


def _engine_worker(rank, world, port, k, result_path):
    """One rank of a 2-rank job on ONE GPU: its shard from the HIP engine."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import pathsim_oracle as po
        from dpathsim.engine import build_engine
        from dpathsim.synth import synth_dblp
        from dpathsim.dist import pack_counts, shard_edges
        from dpathsim.synth import synth_config
        # the bench shape: config3 at 1/20 scale (4 tiles of 16384), engine
        # defaults -- auto W = 16384, venue skipping, companion half tiles
        t = synth_config("config3", scale=0.05).typed()
        eng = build_engine(t, device="cuda:0")
        assert eng.tile_w == 16384 and eng.venue_skip and eng.half_tiles
        na = t.n_authors
        # bench.py's plan: dps_shard_edges over the build's row work (HIP), the
        # same edges as the PyTorch plan over row_work()
        edges = shard_edges(eng.tensor("row_terms")[:na], world)
        e = edges.cpu().tolist()
        bounds = [(e[r], e[r + 1]) for r in range(world)]
        assert bounds == balanced_bounds(eng.row_work(), world)
        mism = torch.zeros(1, dtype=torch.int64, device=eng.device)
        shard_edges(eng.tensor("row_terms")[:na], world, ref=edges, mismatch=mism)
        assert int(mism.item()) == 0
        r0, r1 = bounds[rank]
        m = max_shard(na, world, bounds)
        out = tuple(torch.zeros((m, k), dtype=dt, device=eng.device)
                    for dt in (torch.int32, torch.int64, torch.float64))
        eng.topk(k, r0, r1, out=tuple(o[: r1 - r0] for o in out))
        res = gather_topk(out, na, world, bounds=bounds)
        # bench.py's wire path: 8-byte (count, index) words (dps_pack_counts),
        # rows reordered and rescored on rank 0 (dps_unpack_gathered)
        packed = pack_counts(out[0], out[1])
        res8 = gather_topk_compact(packed, eng.tensor("den")[:na], na, world, bounds=bounds,
                                   edges=edges)
        if rank == 0:
            fi, fc, fs = po.COracle.from_typed(t).topk(k, 0, na)
            ok = True
            for r in (res, res8):
                gi, gc, gs = (a.cpu().numpy() for a in r)
                ok = ok and (np.array_equal(gi, fi) and np.array_equal(gc, fc)
                             and np.array_equal(gs.view(np.int64), fs.view(np.int64)))
            with open(result_path, "w") as f:
                f.write("ok" if ok else "mismatch")
    finally:
        dist.destroy_process_group()


def _tilesplit_cpu_worker(rank, world, port, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dpathsim.dist import TileSplit
        sp = TileSplit.from_group(device="cpu")
        send = torch.arange(5, dtype=torch.int32) + 100 * rank
        recv = torch.empty(5 * world, dtype=torch.int32)
        sp.allgather(send, recv)
        want = torch.cat([torch.arange(5, dtype=torch.int32) + 100 * r for r in range(world)])
        ok = torch.equal(recv, want) and sp.allreduce_max(7 * rank + 1) == 7 * (world - 1) + 1
        ok = ok and (sp.rank, sp.world) == (rank, world)
        flags = torch.tensor([1 if ok else 0], dtype=torch.int64)
        dist.all_reduce(flags, op=dist.ReduceOp.MIN)
        if rank == 0:
            with open(result_path, "w") as f:
                f.write("ok" if int(flags) == 1 else "mismatch")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_tilesplit_collectives_gloo(tmp_path, world):
    """dist.TileSplit's all-gather (rank r's slice at r * size) and the plan's
    max over ranks, over gloo on CPU."""
    out = tmp_path / "result.txt"
    mp.start_processes(_tilesplit_cpu_worker, args=(world, _free_port(), str(out)), nprocs=world,
                       join=True, start_method="spawn")
    assert out.read_text() == "ok"


def _split_worker(rank, world, port, k, result_path):
    """One rank of a 2-rank job on ONE GPU with the N > 1 build's tile split
    (dist.TileSplit over gloo): each rank builds its own target-tile range,
    the slices are all-gathered and assembled; a second build runs with the
    plan's capacities; the assembled tiles equal the single-GPU build's and the
    gathered top-k is the oracle's."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import pathsim_oracle as po
        from dpathsim.dist import TileSplit, pack_counts, shard_edges
        from dpathsim.engine import PathSimEngine, build_engine
        from dpathsim.synth import synth_config
        t = synth_config("config3", scale=0.05).typed()
        na, nv = t.n_authors, t.n_mids
        eng = PathSimEngine(t, device="cuda:0")
        eng.split = TileSplit.from_group(device="cuda:0")
        eng.upload().build()                     # first build + the plan (collective)
        caps = dict(eng.split.caps)
        eng.build()                              # with the plan's capacities
        ok = eng.split.caps == caps and all(v > 0 for v in caps.values())
        ref = build_engine(t, device="cuda:0")
        for w, o_n, m_n in ((16384, "tile_off", "tile_maxc"), (8192, "half_off", "half_maxc")):
            T = -(-na // w)
            ok = ok and torch.equal(ref.tensor(o_n)[: nv * T + 1], eng.tensor(o_n)[: nv * T + 1])
            ok = ok and torch.equal(ref.tensor(m_n)[: nv * T], eng.tensor(m_n)[: nv * T])
        edges = shard_edges(eng.tensor("row_terms")[:na], world)
        e = edges.cpu().tolist()
        bounds = [(e[r], e[r + 1]) for r in range(world)]
        r0, r1 = bounds[rank]
        m = max_shard(na, world, bounds)
        out = tuple(torch.zeros((m, k), dtype=dt, device=eng.device)
                    for dt in (torch.int32, torch.int64, torch.float64))
        eng.topk(k, r0, r1, out=tuple(o[: r1 - r0] for o in out))
        res = gather_topk_compact(pack_counts(out[0], out[1]), eng.tensor("den")[:na], na, world,
                                  bounds=bounds, edges=edges)
        flags = torch.tensor([1 if ok else 0], dtype=torch.int64)
        dist.all_reduce(flags, op=dist.ReduceOp.MIN)
        if rank == 0:
            fi, fc, fs = po.COracle.from_typed(t).topk(k, 0, na)
            gi, gc, gs = (a.cpu().numpy() for a in res)
            good = (int(flags) == 1 and np.array_equal(gi, fi) and np.array_equal(gc, fc)
                    and np.array_equal(gs.view(np.int64), fs.view(np.int64)))
            with open(result_path, "w") as f:
                f.write("ok" if good else f"mismatch (tiles {int(flags)})")
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_gloo_two_ranks_split_tile_build(tmp_path):
    out = tmp_path / "result.txt"
    mp.start_processes(_split_worker, args=(2, _free_port(), 10, str(out)), nprocs=2,
                       join=True, start_method="spawn")
    assert out.read_text() == "ok"


@pytest.mark.gpu
def test_gloo_two_ranks_engine_shards(tmp_path):
    out = tmp_path / "result.txt"
    mp.start_processes(_engine_worker, args=(2, _free_port(), 10, str(out)), nprocs=2,
                       join=True, start_method="spawn")
    assert out.read_text() == "ok"


def _rccl_worker(rank, world, port, k, result_path):
    """The compact gather on the nccl (RCCL) backend with one rank: the same
    dist.gather call bench.py makes at N > 1 (a one-GPU box cannot host two
    RCCL ranks)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world)
    try:
        import pathsim_oracle as po
        from dpathsim.dist import pack_counts
        from dpathsim.engine import build_engine
        from dpathsim.synth import synth_dblp
        t = synth_dblp(4000, 12000, 200, seed=8).typed()
        eng = build_engine(t, device="cuda:0")
        na = t.n_authors
        idx, cnt, _ = eng.topk(k)
        out = torch.empty((na, k), dtype=torch.int64, device="cuda:0")
        gi, gc, gs = gather_topk_compact(pack_counts(idx, cnt), eng.tensor("den")[:na], na, 1,
                                         out=out, force_collective=True)
        fi, fc, fs = po.COracle.from_typed(t).topk(k, 0, na)
        ok = (np.array_equal(gi.cpu().numpy(), fi) and np.array_equal(gc.cpu().numpy(), fc)
              and np.array_equal(gs.cpu().numpy().view(np.int64), fs.view(np.int64)))
        with open(result_path, "w") as f:
            f.write("ok" if ok else "mismatch")
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_rccl_compact_gather_one_rank(tmp_path):
    out = tmp_path / "result.txt"
    mp.start_processes(_rccl_worker, args=(1, _free_port(), 10, str(out)), nprocs=1,
                       join=True, start_method="spawn")
    assert out.read_text() == "ok"


def _rccl_capi_worker(rank, world, port, k, result_path):
    """The compact gather through libdpathsim's own RCCL communicator
    (dps_comm_init / dps_gather / dps_bcast; torch.distributed gloo only
    carries the unique id), one rank -- bench.py's N > 1 wire path."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = None
    try:
        import pathsim_oracle as po
        from dpathsim.dist import RcclComm, check_comm_gather, pack_counts
        from dpathsim.engine import build_engine
        from dpathsim.synth import synth_dblp
        comm = RcclComm()
        # bench.py's pre-loop known-pattern check through the real communicator
        if not check_comm_gather(comm, "cuda:0"):
            raise AssertionError("check_comm_gather failed through RcclComm")
        t = synth_dblp(4000, 12000, 200, seed=8).typed()
        eng = build_engine(t, device="cuda:0")
        na = t.n_authors
        idx, cnt, _ = eng.topk(k)
        out = torch.empty((na, k), dtype=torch.int64, device="cuda:0")
        gi, gc, gs = gather_topk_compact(pack_counts(idx, cnt), eng.tensor("den")[:na], na, 1,
                                         out=out, force_collective=True, comm=comm)
        fi, fc, fs = po.COracle.from_typed(t).topk(k, 0, na)
        ok = (np.array_equal(gi.cpu().numpy(), fi) and np.array_equal(gc.cpu().numpy(), fc)
              and np.array_equal(gs.cpu().numpy().view(np.int64), fs.view(np.int64)))
        b = torch.arange(1000, dtype=torch.int64, device="cuda:0")
        comm.bcast(b)
        ok = ok and bool((b.cpu() == torch.arange(1000)).all())
        with open(result_path, "w") as f:
            f.write("ok" if ok else "mismatch")
    finally:
        if comm is not None:
            comm.close()
        dist.destroy_process_group()


@pytest.mark.gpu
def test_rccl_capi_compact_gather_one_rank(tmp_path):
    out = tmp_path / "result.txt"
    mp.start_processes(_rccl_capi_worker, args=(1, _free_port(), 10, str(out)), nprocs=1,
                       join=True, start_method="spawn")
    assert out.read_text() == "ok"


def test_read_topk_shards_rejects_stale_or_mixed(tmp_path):
    """A shard directory whose manifests do not start at row 0, disagree on k,
    or whose arrays do not match their manifest is refused, not merged."""
    import json
    from dpathsim.dist import write_topk_shard
    k = 3
    parts = [tuple(torch.zeros((n, k), dtype=dt) for dt in (torch.int32, torch.int64, torch.float64))
             for n in (4, 6)]
    bounds = [(0, 4), (4, 10)]
    for r in range(2):
        write_topk_shard(str(tmp_path), r, 2, bounds, parts[r], k)
    assert read_topk_shards(str(tmp_path))[0].shape == (10, k)
    m1 = tmp_path / "topk_rank00001.json"
    meta = json.loads(m1.read_text())
    m1.write_text(json.dumps(dict(meta, k=4)))
    with pytest.raises(ValueError, match="k"):
        read_topk_shards(str(tmp_path))
    m1.write_text(json.dumps(meta))
    np.save(tmp_path / "topk_rank00001.npy", np.zeros((5, 2 * k), np.int64))
    with pytest.raises(ValueError, match="shape"):
        read_topk_shards(str(tmp_path))
    m0 = tmp_path / "topk_rank00000.json"
    meta0 = json.loads(m0.read_text())
    m0.write_text(json.dumps(dict(meta0, row_begin=1)))
    with pytest.raises(ValueError, match="row 0"):
        read_topk_shards(str(tmp_path))


class _GlooComm:
    """A stand-in for dist.RcclComm over the gloo group (CPU tensors): a true
    gather, a corrupting one, or one that raises."""

    def __init__(self, mode):
        self.rank, self.world, self.mode = dist.get_rank(), dist.get_world_size(), mode

    def gather(self, send, recv, root=0):
        parts = [torch.empty_like(send) for _ in range(self.world)] if self.rank == root else None
        dist.gather(send, gather_list=parts, dst=root)
        if self.mode == "raise" and self.rank == 1:      # an error status after the call
            raise RuntimeError("simulated dps_gather failure")
        if self.rank == root:
            recv.copy_(torch.cat(parts))
            if self.mode == "corrupt":
                recv[-1] += 1


def _comm_check_worker(rank, world, port, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dpathsim.dist import check_comm_gather
        got = [check_comm_gather(_GlooComm(m), "cpu") for m in ("good", "corrupt", "raise")]
        if rank == 0:
            with open(result_path, "w") as f:
                f.write(",".join(str(g) for g in got))
        else:
            with open(f"{result_path}.{rank}", "w") as f:
                f.write(",".join(str(g) for g in got))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_check_comm_gather_verdict_on_every_rank(tmp_path, world):
    """bench.py's pre-timing check of the C-ABI gather: a true
    gather passes, a corrupted or failing one fails -- and every rank gets the
    same verdict, so all of them take the same gather path."""
    out = tmp_path / "result.txt"
    mp.start_processes(_comm_check_worker, args=(world, _free_port(), str(out)), nprocs=world,
                       join=True, start_method="spawn")
    assert out.read_text() == "True,False,False"
    for r in range(1, world):
        assert (tmp_path / f"result.txt.{r}").read_text() == "True,False,False"


def _comm_id_fail_worker(rank, world, port, result_path):
    """RcclComm when rank 0 cannot create the RCCL unique id: the failure is
    broadcast with the id's bytes, so every rank raises instead of waiting."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dpathsim import _lib
        from dpathsim.dist import RcclComm
        real = _lib.call

        def call(name, *a):
            if name == "dps_comm_get_id":
                raise _lib.DPSError(name, _lib.DPS_ERR_HIP, "simulated ncclGetUniqueId failure")
            if name == "dps_comm_init":
                raise AssertionError("dps_comm_init reached after a failed unique id")
            return real(name, *a)
        _lib.call = call
        try:
            RcclComm(device="cpu")
            msg = "no error"
        except RuntimeError as e:
            msg = "raised" if "dps_comm_get_id failed on rank 0" in str(e) else f"other: {e}"
        with open(f"{result_path}.{rank}", "w") as f:
            f.write(msg)
    finally:
        dist.destroy_process_group()


def test_rccl_comm_id_failure_reaches_every_rank(tmp_path):
    out = tmp_path / "result.txt"
    mp.start_processes(_comm_id_fail_worker, args=(2, _free_port(), str(out)), nprocs=2,
                       join=True, start_method="spawn")
    assert [open(f"{out}.{r}").read() for r in range(2)] == ["raised", "raised"]
