#!/usr/bin/env python3
"""Benchmark: APVPA all-pairs PathSim top-k, scored pairs/s (BASELINE.json metric).

One "step" = the whole hot path over one synthetic graph already resident in
HBM: typed incidence extraction -> typed CSR build (distinct) -> SpGEMM C ->
s, g -> target-tiled C^T -> fused C.C^T + fp64 score + top-k over this rank's
author rows -> gather of every rank's top-k to rank 0 (one RCCL gather of
8-byte (count, index) words; rank 0 rescores with its own g).
value = N_A*(N_A-1) / step time (max over ranks), whole job.

Workload (configs[1] = dblp_large.gexf is absent, .MISSING_LARGE_BLOBS:1):
BASELINE.json configs[2] "synthetic DBLP-shaped graph (1M authors, 3M papers,
5k venues) APVPA top-10, row-sharded at 1/2/4/8 GPUs" -- dpathsim.synth
config3, seed 20180417.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config config3]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "distributed-pathsim_amd"))

CLK_GHZ, N_CU = 2.4, 256
# LDS bytes per clock per CU by instruction class (MI355X_MICROARCH.md §LDS):
LDS_READ_B128 = 256.0    # ds_read_b128 (the accumulator read)
LDS_WRITE_B128 = 79.0    # ds_write_b128 (zeroing the accumulator)
LDS_ADD_B32 = 64.0       # ds_add_u32 = a b32-class store (the scatter)
LDS_PEAK_GBS = LDS_READ_B128 * N_CU * CLK_GHZ   # b128-read-equivalent peak, GB/s
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="config3")
    ap.add_argument("--scale", type=float, default=1.0, help="shrink authors/papers (debug)")
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--tile-w", type=int, default=None,
                    help="target tile width (default: the engine's choice by shape)")
    ap.add_argument("--denominator", default="rowsum", choices=["rowsum", "diag"])
    ap.add_argument("--venue-skip", type=int, default=None,
                    help="1/0: force venue skipping on/off (default: the engine's)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pmc-json", default=os.path.join(REPO, "profiles", "r06", "pmc_hot.json"),
                    help="rocprofv3 PMC summary of the hot kernel at HEAD (tools/pmc_hot.py): "
                         "HBM bytes per launch (roofline.traffic) and VALU issue share")
    return ap.parse_args()


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    from dpathsim.dist import (RcclComm, TileSplit, check_comm_gather, gather_topk_compact,
                               max_shard, pack_counts, shard_edges)
    from dpathsim.engine import PathSimEngine
    from dpathsim.synth import CONFIGS, synth_config

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs for the multi-rank path on a one-GPU box (never set by the
    # driver): all ranks on one device, the gather over gloo instead of RCCL
    local = int(os.environ.get("DPATHSIM_BENCH_DEVICE", local))
    backend = os.environ.get("DPATHSIM_BENCH_BACKEND", "rccl")
    # the top-k gather over RCCL (xGMI): by default through libdpathsim's C ABI
    # (dps_comm_init / dps_gather = ncclCommInitRank / RCCL send-recv on the
    # step's stream; gloo is only the control plane: the unique id, barriers,
    # the timing max) -- SURVEY 8b's dps_gather.  Before the
    # timed loop rank 0 checks one gather of a known pattern through it in this
    # process; on a mismatch (or an error) every rank switches to a
    # torch.distributed nccl group for the gather, in the same process.
    # DPATHSIM_BENCH_COMM=torch uses the nccl process group from the start.
    comm_kind = os.environ.get("DPATHSIM_BENCH_COMM", "capi")
    comm = None
    gather_group = None          # the torch group of the gather when comm is None
    comm_used = "none" if world == 1 else backend
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1:
        if backend == "rccl" and comm_kind == "torch":
            dist.init_process_group("nccl", device_id=dev)
            comm_used = "torch-nccl"
        else:
            dist.init_process_group("gloo")
            if backend == "rccl":
                try:
                    comm = RcclComm(device=dev)
                except Exception as e:    # noqa: BLE001 -- falls back below, on every rank
                    print(f"rank {rank}: dps_comm_init failed ({e})", file=sys.stderr)
                    comm = None
                # every rank takes the same branch: the check is a collective
                up = torch.tensor([0 if comm is None else 1], dtype=torch.int64)
                dist.all_reduce(up, op=dist.ReduceOp.MIN)
                if int(up.item()) == 1 and check_comm_gather(comm, dev):
                    comm_used = "capi-rccl"
                else:
                    if comm is not None:
                        comm.close()
                    comm = None
                    if rank == 0:
                        print("the C-ABI RCCL gather failed its known-pattern check: "
                              "using torch.distributed's nccl group", file=sys.stderr)
                    gather_group = dist.new_group(backend="nccl")
                    comm_used = "torch-nccl (C-ABI check failed)"

    na_cfg, np_cfg, nm_cfg, mp_name, k_cfg = CONFIGS[args.config]
    k = args.k or k_cfg
    graph = synth_config(args.config, scale=args.scale)
    typed = graph.typed(__import__("dpathsim").METAPATHS[mp_name])
    NA = typed.n_authors

    eng = PathSimEngine(typed, device=dev, tile_w=args.tile_w,
                        denominator=args.denominator)
    args.tile_w = eng.tile_w
    if args.venue_skip is not None:
        eng.venue_skip = bool(args.venue_skip) and args.denominator == "rowsum"
    # N > 1: DPATHSIM_BENCH_SPLIT=1 -- each rank builds the C^T tiles of its own
    # target-tile range and the slices are all-gathered (dist.TileSplit,
    # DESIGN.md §10); C, g and the target order stay replicated.  Off by
    # default: on one GPU the per-rank slice build measured 1.70-1.77 ms against
    # 2.0 ms for the whole build, and the all-gather of the padded slices (63 MB
    # on config3 at N = 8) costs more than that saves (tools/split_balance.py,
    # profiles/r05/split_balance.txt)
    if world > 1 and os.environ.get("DPATHSIM_BENCH_SPLIT", "0") == "1":
        eng.split = TileSplit.from_group(group=gather_group, comm=comm, device=dev)
    eng.upload()

    eng.build()             # checks the overflow conditions once (one sync); with the
                            # tile split also the gather plan (one collective)
    # contiguous row shards of equal estimated work (dps_shard_edges over the
    # build's row work; every rank derives the same edges from its own,
    # identical C: no communication), read back once, outside the timed loop
    edges0 = shard_edges(eng.tensor("row_terms")[:NA], world)
    e_host = edges0.cpu().tolist()
    bounds0 = [(e_host[r], e_host[r + 1]) for r in range(world)]
    m = max_shard(NA, world, bounds0)
    out = (torch.empty((m, k), dtype=torch.int32, device=dev),
           torch.empty((m, k), dtype=torch.int64, device=dev),
           torch.empty((m, k), dtype=torch.float64, device=dev))
    packed = torch.empty((m, k), dtype=torch.int64, device=dev)
    gathered = final = None
    if world > 1 and rank == 0:
        gathered = torch.empty((world * m, k), dtype=torch.int64, device=dev)
        final = (torch.empty((NA, k), dtype=torch.int32, device=dev),
                 torch.empty((NA, k), dtype=torch.int64, device=dev),
                 torch.empty((NA, k), dtype=torch.float64, device=dev))

    ev_topk = []
    # every step re-derives the shards from its own C on the device (no host
    # read-back inside the step); the launch uses the shards of the first build
    # and any difference is raised after the timed loop
    edges_step = torch.empty_like(edges0)
    plan_mismatch = torch.zeros(1, dtype=torch.int64, device=dev)

    def step(record):
        eng.build(check=False)   # no host read-back inside the step; checked after timing
        if world > 1:
            shard_edges(eng.tensor("row_terms")[:NA], world, out=edges_step, ref=edges0,
                        mismatch=plan_mismatch)
        r0, r1 = bounds0[rank]
        bounds = bounds0
        view = tuple(t[:r1 - r0] for t in out)
        if record:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
        eng.topk(k, r0, r1, out=view)
        if record:
            e1.record()
            ev_topk.append((e0, e1))
        if world > 1:   # one packed buffer per rank, gathered to rank 0 (RCCL)
            # 8 B per slot on the wire: (count << 32) | index (dps_pack_counts);
            # rank 0 puts the rows in order and rebuilds the fp64 scores from its
            # own g with the same exact division (dps_unpack_gathered)
            pack_counts(out[0], out[1], out=packed)
            gather_topk_compact(packed, eng.tensor("den")[:NA], NA, world, group=gather_group,
                                out=gathered, bounds=bounds, comm=comm, edges=edges0,
                                result=final)

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    eng.check()              # the last step's overflow conditions (raises if violated)
    if int(plan_mismatch.item()) != 0:
        raise RuntimeError("row shards changed between steps")
    if world > 1:
        te = torch.tensor([elapsed], dtype=torch.float64,
                          device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
        elapsed = float(te.item())
    ms_per_step = elapsed * 1e3 / args.steps
    pairs = NA * (NA - 1)
    value = pairs / (elapsed / args.steps)

    # ---- roofline of the dominant kernel (dps_cct_topk -> k_cct1), measured live --
    # ALGORITHMIC work of one launch (the SIMT path's unit is one
    # term C[x,v]*C[y,v], sum_{x in shard} sum_{v in x} n_v of them), priced on the
    # LDS per instruction class (MI355X_MICROARCH.md §LDS):
    #   scatter  one ds_add_u32 per term, 4 B (b32 store class, 64 B/clk/CU);
    #   read     the packed counters of every (row, target) pair once, 1/2 B per
    #            pair at 4-bit counters (tile_w 16384), 1 B at u8 (ds_read_b128,
    #            256 B/clk/CU);
    #   zero     the same bytes rewritten (ds_write_b128, 79 B/clk/CU);
    # floor = sum of bytes / rate / (256 CUs x 2.4 GHz); frac = floor / launch time
    # (events on the kernel's stream).  `achieved` / `peak` express the same in
    # b128-read-equivalent bytes.  This work is fixed by the problem: venue and
    # tile skipping do less of it (the executed counts -- passes, chunks -- are
    # reported beside it, with their own floor), which shows as a higher frac.
    # HBM (secondary, logical): 2 B per term (16-bit C^T entries) + 20 B per
    # output slot + row offsets; `traffic` = PMC bytes of the same launch.
    topk_ms = float(np.mean([a.elapsed_time(b) for a, b in ev_topk]))
    r0, r1 = bounds0[rank]
    shard = r1 - r0
    c_ptr = eng.tensor("c_ptr")
    nnz = eng.info.nnz_c
    c_col = eng.tensor("c_col")[:nnz].long()
    n_v = torch.bincount(c_col, minlength=typed.n_mids)
    w = torch.zeros(nnz + 1, dtype=torch.int64, device=dev)
    w[1:] = torch.cumsum(n_v[c_col], 0)
    terms = int((w[c_ptr[r1]] - w[c_ptr[r0]]).item())      # sum_{x in shard} sum_{v in x} n_v
    ent_bytes = 2 if args.tile_w <= 16384 else 4
    kc = eng.kernel_counts()                         # the last launch's counts
    n_pass, n_chunk, n_ver = kc["passes"], kc["chunks"], kc["verified"]
    bytes_launch = ent_bytes * terms + 20 * shard * k + 8 * (shard + 1)
    hbm_achieved = bytes_launch / (topk_ms * 1e-3) / 1e9
    ctr_bytes = 0.5 if args.tile_w in (16384, 15360) else 1.0 if args.tile_w <= 8192 else 4.0
    acc_bytes = 7680 if args.tile_w in (7680, 15360) else 8192   # one pass's accumulator
    pairs_launch = shard * (NA - 1)
    lds_rate = {"scatter_add_b32": LDS_ADD_B32, "acc_read_b128": LDS_READ_B128,
                "acc_zero_b128": LDS_WRITE_B128}

    def lds_price(cls):
        floor = {c: b / lds_rate[c] / (N_CU * CLK_GHZ * 1e9) * 1e3 for c, b in cls.items()}
        equiv = sum(b * LDS_READ_B128 / lds_rate[c] for c, b in cls.items())
        return floor, equiv

    lds_cls = {"scatter_add_b32": 4 * terms, "acc_read_b128": int(ctr_bytes * pairs_launch),
               "acc_zero_b128": int(ctr_bytes * pairs_launch)}
    lds_floor_ms, lds_equiv = lds_price(lds_cls)
    lds_bytes = sum(lds_cls.values())
    lds_achieved = lds_equiv / (topk_ms * 1e-3) / 1e9
    # executed: what the kernel counted (k_cct1 only: 16-byte chunks scattered, 8 KiB
    # accumulator passes read and zeroed)
    exe_cls = {"scatter_add_b32": 32 * n_chunk, "acc_read_b128": acc_bytes * n_pass,
               "acc_zero_b128": acc_bytes * n_pass}
    exe_floor_ms, _ = lds_price(exe_cls)
    traffic, pmc = None, {}
    if args.pmc_json and os.path.exists(args.pmc_json):
        try:
            pm = json.load(open(args.pmc_json))
            if (pm.get("config") == args.config and pm.get("world", 1) == world
                    and pm.get("tile_w", args.tile_w) == args.tile_w and args.scale == 1.0
                    and pm.get("k", k) == k and args.denominator == "rowsum"
                    and pm.get("venue_skip", False) == bool(eng._ext is not None and eng._ext.s)):
                traffic = pm.get("hbm_bytes_per_launch")
                pmc = {key: pm.get(key) for key in ("lds", "valu", "wait")}
        except Exception:
            traffic, pmc = None, {}
    info = eng.info

    # ---- secondary rates the north star asks for -----------------------------
    # SpGEMM (C = W_AP . W_PV) against HBM: SURVEY §8d algorithmic bytes over the
    # 'spgemm' phase of one extra timed build (events on the stream).
    eng.build(timed=True)
    sp_ms = eng.info.phase_ms.get("spgemm", float("nan"))
    sp_bytes = (16 * (NA + 1) + 8 * eng.info.nnz_ap + 4 * typed.n_papers + 8 * eng.info.nnz_c)
    spgemm = {"bound": "hbm", "phase_ms": sp_ms, "algorithmic_bytes": sp_bytes,
              "achieved": sp_bytes / (sp_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s"}
    spgemm["frac"] = spgemm["achieved"] / HBM_PEAK_GBS
    # C.C^T against the dense int8 MFMA peak (5 POPS, MI355X_MICROARCH.md): the
    # intrinsic sparse rate (2 * sum_{x in shard} sum_{v in x} n_v multiply-adds)
    # as a fraction of that peak, and -- as a rate, not a fraction -- the
    # dense-equivalent ops/s (2 * rows * N_A * V padded to 64) the all-pairs
    # product would need on MFMA to finish in the same time.
    v_pad = (typed.n_mids + 63) // 64 * 64
    cct = {"mfma_int8_dense_peak_ops": 5.0e15,
           "intrinsic_ops_per_s": 2.0 * terms / (topk_ms * 1e-3),
           "dense_equiv_ops_per_s": 2.0 * shard * NA * v_pad / (topk_ms * 1e-3)}
    cct["intrinsic_frac_of_mfma_int8_peak"] = cct["intrinsic_ops_per_s"] / 5.0e15

    # ---- PCIe-inclusive rate (not `value`): the boundary takes host arrays
    # (edge list + node tables, engine.upload); time their host -> HBM copies
    # (pageable numpy memory, as a caller hands them over) and add them to a step.
    h2d_arrays = [graph.edge_src, graph.edge_dst, typed.edge_rel, typed.node_type,
                  typed.node_rowid, typed.node_colid]
    h2d_bytes = int(sum(a.nbytes for a in h2d_arrays))
    h2d = []
    for _ in range(3):
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        held = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in h2d_arrays]
        torch.cuda.synchronize(dev)
        h2d.append((time.perf_counter() - t1) * 1e3)
        del held
    h2d_ms = float(np.median(h2d))
    # the same copies from pinned (page-locked) host buffers, as a caller that
    # stages its edge list for the GPU would hand them over
    pinned = [torch.from_numpy(np.ascontiguousarray(a)).pin_memory() for a in h2d_arrays]
    h2d_p = []
    for _ in range(3):
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        held = [a.to(dev, non_blocking=True) for a in pinned]
        torch.cuda.synchronize(dev)
        h2d_p.append((time.perf_counter() - t1) * 1e3)
        del held
    del pinned
    h2d_pin_ms = float(np.median(h2d_p))
    pcie = {"h2d_bytes": h2d_bytes, "h2d_ms": h2d_ms, "h2d_GBps": h2d_bytes / (h2d_ms * 1e-3) / 1e9,
            "value_incl_h2d": pairs / ((ms_per_step + h2d_ms) * 1e-3),
            "h2d_pinned_ms": h2d_pin_ms,
            "h2d_pinned_GBps": h2d_bytes / (h2d_pin_ms * 1e-3) / 1e9,
            "value_incl_h2d_pinned": pairs / ((ms_per_step + h2d_pin_ms) * 1e-3),
            "note": "SURVEY 8d's host-resident variant: the edge list + node tables copied "
                    "host -> HBM each step (pageable, and pinned); not the reported value"}

    # ---- CPU baseline: the oracle's C port on a bounded row sample ----------
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        try:
            import pathsim_oracle as po
            threads = os.cpu_count() or 1
            threads = min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))
            co = po.COracle.from_typed(typed)
            co.topk(k, 0, 64, threads=threads)          # warm-up: per-thread accumulators
            rows, dt, chunk = 0, 0.0, 256
            while dt < args.cpu_baseline_seconds and rows < NA:   # doubling row blocks
                n = min(chunk, NA - rows)
                t1 = time.perf_counter()
                co.topk(k, rows, rows + n, threads=threads)
                dt += time.perf_counter() - t1
                rows += n
                chunk *= 2
            cpu = {"value": rows * (NA - 1) / dt, "unit": "pairs/s", "cores": threads,
                   "kind": "port",
                   "sample": f"oracle/pathsim_oracle.c (OpenMP), author rows [0,{rows}) x all "
                             f"{NA} targets of {args.config}, top-{k}, {dt:.1f} s; reference "
                             "Spark/graphframes unavailable (no JVM/pyspark; log: 0.00894 pairs/s)"}
        except Exception as e:  # pragma: no cover
            cpu = {"value": None, "unit": "pairs/s", "cores": 0, "kind": "port",
                   "sample": f"unavailable: {e}"}

    if rank == 0:
        rec = {
            "metric": f"PathSim pairs scored/sec ({mp_name} all-pairs top-k)",
            "value": value,
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int32+f64",
            "denominator": args.denominator,
            "data": "synthetic (dpathsim.synth, seed 20180417; dblp_large.gexf is absent)",
            "config": {"workload": f"{args.config}: synthetic DBLP {mp_name} "
                                   f"{NA} authors / {typed.n_papers} papers / "
                                   f"{typed.n_mids} {typed.metapath.mid_type}s, all-pairs top-{k}",
                       "n_authors": NA, "k": k, "tile_w": args.tile_w,
                       "nnz_C": info.nnz_c, "sum_terms": terms if world == 1 else None,
                       "inputs": "edge list + node tables resident in HBM when the timed "
                                 "region starts (the bench contract); SURVEY 8d times them "
                                 "host-resident: that rate is pcie_inclusive.value_incl_h2d*",
                       "parallelism": f"row-shard x{world} (work-balanced, heaviest rows first)",
                       "gather": comm_used,
                       "build": ("C^T tiles split by target-tile range + all-gather"
                                 if eng.split is not None else "replicated")},
            # bound: the LDS array (the resource the algorithm's unit work lands on;
            # the kernel itself is issue/latency-bound at the occupancy its LDS
            # allows)
            "roofline": {"bound": "lds", "kernel": f"dps_cct_topk (k_cct1, W {args.tile_w})",
                         "achieved": lds_achieved, "peak": LDS_PEAK_GBS,
                         "unit": "GB/s (ds_read_b128-equivalent)",
                         "frac": lds_achieved / LDS_PEAK_GBS,
                         "traffic": traffic,
                         "lds_bytes": lds_bytes, "lds_bytes_by_class": lds_cls,
                         "lds_rate_B_per_clk_cu": lds_rate,
                         "lds_floor_ms_by_class": lds_floor_ms,
                         "lds_floor_ms": sum(lds_floor_ms.values()),
                         "executed": {"passes": n_pass, "chunks": n_chunk, "verified": n_ver,
                                      "lds_bytes_by_class": exe_cls,
                                      "lds_floor_ms": sum(exe_floor_ms.values()) if n_pass else None,
                                      "frac": (sum(exe_floor_ms.values()) / topk_ms) if n_pass else None},
                         "venue_skip": bool(eng._ext is not None and eng._ext.s),
                         "half_tiles": bool(eng._ext is not None and eng._ext.half_ent),
                         "avg_launch_ms": topk_ms,
                         "pmc": pmc,
                         "hbm": {"algorithmic_bytes": bytes_launch,
                                 "achieved": hbm_achieved, "peak": HBM_PEAK_GBS,
                                 "frac": hbm_achieved / HBM_PEAK_GBS,
                                 "traffic_frac": (traffic / (topk_ms * 1e-3) / 1e9 / HBM_PEAK_GBS)
                                 if traffic else None}},
            "cpu_baseline": cpu,
            "phases_ms": {"cct_topk": topk_ms, "rest_of_step": ms_per_step - topk_ms},
            "pcie_inclusive": pcie,
            "spgemm_roofline": spgemm,
            "cct_vs_mfma": cct,
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.barrier()
        if comm is not None:
            comm.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
