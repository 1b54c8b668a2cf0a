"""Command line of the engine: ``python -m dpathsim`` (SURVEY.md §5 "Config / flags").

The reference hard-codes its inputs (DPathSim_APVPA.py:141-142 graph path,
:171 source author "Jiawei Han", :175-176 the log path
``output/d_pathsim_output_%Y%m%d_%H%M%S.log`` in gmtime) and runs one source
against every author.  The flags replace those constants:

  single source (the reference's run(), same prints and log lines):
    python -m dpathsim --graph dblp/dblp_small.gexf --source-name "Some Author"

  all-pairs top-k (the build's generalisation, native log writer):
    python -m dpathsim --graph G.gexf --all-pairs --topk 10 [--denominator diag]
    python -m dpathsim --synth config3 --all-pairs --topk 10 --out run.log
    torchrun --nproc-per-node 8 -m dpathsim --synth config5 --all-pairs --topk 100 \
        --shard-dir out/       # per-rank shard files instead of one gathered log

``--denominator rowsum`` (default) is the reference's global-walk row sum
(SURVEY K2); ``diag`` is the textbook PathSim M[x,x] + M[y,y].  ``--gpus N``
under torchrun shards the author rows over N ranks (one GPU each, RCCL);
without torchrun it must be 1.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def parse(argv=None):
    ap = argparse.ArgumentParser(prog="python -m dpathsim", description=__doc__.split("\n")[0])
    src = ap.add_mutually_exclusive_group(required=True)
    src.add_argument("--graph", help="GEXF file (the reference's dblp/*.gexf layout)")
    src.add_argument("--synth", help="synthetic graph: config3, config3_100k, config4, config5")
    ap.add_argument("--scale", type=float, default=1.0, help="shrink a --synth graph")
    ap.add_argument("--metapath", default="APVPA", help="APVPA (default) or APTPA")
    mode = ap.add_mutually_exclusive_group()
    mode.add_argument("--source-name", help="single-source run() for the author with this label")
    mode.add_argument("--all-pairs", action="store_true", help="all-pairs top-k")
    ap.add_argument("--topk", type=int, default=10)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--denominator", default="rowsum", choices=["rowsum", "diag"])
    ap.add_argument("--tile-w", type=int, default=None,
                    help="target tile width (default: the engine's choice by shape)")
    ap.add_argument("--out", help="log path (default: output/d_pathsim_output_<gmtime>.log)")
    ap.add_argument("--shard-dir", help="all-pairs: write per-rank shard files here instead "
                                        "of gathering to rank 0")
    ap.add_argument("--metrics-json", help="append one JSON metrics record to this file")
    ap.add_argument("--quiet", action="store_true", help="no per-target stdout (single source)")
    a = ap.parse_args(argv)
    if not a.source_name and not a.all_pairs:
        ap.error("choose --source-name NAME (single source) or --all-pairs")
    if a.source_name and a.denominator != "rowsum":
        ap.error("--denominator diag applies to --all-pairs (run() keeps the reference's row sums)")
    if a.topk < 1 or a.topk > 256:
        ap.error("--topk must be in [1, 256]")
    return a


def _default_log_path():
    # DPathSim_APVPA.py:175-176: gmtime-stamped file under output/
    return "output/d_pathsim_output_{}.log".format(time.strftime("%Y%m%d_%H%M%S", time.gmtime()))


def _load(a):
    from .compat import read_dblp_nx_file
    from .graph import METAPATHS
    from .synth import synth_config
    mp = METAPATHS[a.metapath]
    t0 = time.perf_counter()
    if a.graph:
        g, _, _ = read_dblp_nx_file(a.graph)
    else:
        g = synth_config(a.synth, scale=a.scale)
    return g, mp, time.perf_counter() - t0


def main(argv=None):
    a = parse(argv)
    import torch

    from .compat import DPathSim_APVPA, find_author_node_id_by_name
    from .engine import build_engine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world:
        raise SystemExit(f"--gpus {a.gpus} needs a torchrun launch with {a.gpus} processes "
                         f"(WORLD_SIZE is {world})")
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    graph, mp, load_s = _load(a)
    typed = graph.typed(mp)
    out_path = a.out or _default_log_path()
    if os.path.dirname(out_path):
        os.makedirs(os.path.dirname(out_path), exist_ok=True)
    metrics = {"graph": a.graph or a.synth, "metapath": mp.name, "n_authors": typed.n_authors,
               "load_s": load_s, "denominator": a.denominator}

    if a.source_name:
        if world > 1:
            raise SystemExit("single-source mode runs on one GPU")
        src = find_author_node_id_by_name(graph, a.source_name)     # :171-172 (None if absent)
        t0 = time.perf_counter()
        eng = build_engine(typed, device=dev, tile_w=a.tile_w)
        job = DPathSim_APVPA(graph, eng, src, out_path)
        if a.quiet:
            import contextlib
            import io
            with contextlib.redirect_stdout(io.StringIO()):
                job.run()
        else:
            job.run()
        metrics.update(mode="single_source", source=src, seconds=time.perf_counter() - t0,
                       log=out_path)
    else:
        from .dist import (balanced_bounds, gather_topk, max_shard, pack_topk,
                           write_topk_shard)
        from .logfmt import write_topk_log
        k = a.topk
        t0 = time.perf_counter()
        eng = build_engine(typed, device=dev, tile_w=a.tile_w, denominator=a.denominator)
        na = typed.n_authors
        bounds = balanced_bounds(eng.row_work(), world) if world > 1 else [(0, na)]
        r0, r1 = bounds[rank]
        m = max_shard(na, world, bounds)
        out = tuple(torch.zeros((m, k), dtype=dt, device=dev)
                    for dt in (torch.int32, torch.int64, torch.float64))
        eng.topk(k, r0, r1, out=tuple(o[: r1 - r0] for o in out))
        torch.cuda.synchronize(dev)
        compute_s = time.perf_counter() - t0
        # the log's "global walk" lines print the global walk g (the reference's
        # metapath_global_walk, DPathSim_APVPA.py:30,46) whatever the denominator
        walks = eng.tensor("g")[:na].cpu().numpy()
        pairs = max(na - 1, 0) * (r1 - r0)
        per_pair = compute_s / max(pairs, 1)
        t1 = time.perf_counter()
        if a.shard_dir:
            write_topk_shard(a.shard_dir, rank, world, bounds, pack_topk(*out), k)
            metrics["shard_dir"] = a.shard_dir
        else:
            res = gather_topk(pack_topk(*out), na, world, bounds=bounds) if world > 1 else \
                tuple(o[: r1 - r0] for o in out)
            if rank == 0:
                idx, cnt, sc = (t.cpu().numpy() for t in res)
                write_topk_log(out_path, typed, idx, cnt, sc, walks, append=True,
                               stage_seconds=per_pair,
                               overall_seconds=time.perf_counter() - t0)
                metrics["log"] = out_path
        metrics.update(mode="all_pairs", k=k, world=world, compute_s=compute_s,
                       pairs_per_s=na * max(na - 1, 0) / compute_s if compute_s else None,
                       write_s=time.perf_counter() - t1)
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
            dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(metrics), file=sys.stderr, flush=True)
        if a.metrics_json:
            with open(a.metrics_json, "a") as f:
                f.write(json.dumps(metrics) + "\n")
    return 0
