"""Row sharding of the all-pairs top-k across ranks.

Every source row's top-k depends only on that row of C plus all of C and g,
so ranks split the author rows into contiguous, balanced shards and exchange
nothing but the finished top-k blocks.  One process per GPU; the collective is
RCCL (``nccl`` backend) on the GPU box and gloo in the CPU tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_bounds(n_rows: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous balanced shard [r0, r1) of rank ``rank`` out of ``world``."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    return n_rows * rank // world, n_rows * (rank + 1) // world


def max_shard(n_rows: int, world: int, bounds=None) -> int:
    if bounds is None:
        bounds = [shard_bounds(n_rows, r, world) for r in range(world)]
    return max(b - a for a, b in bounds)


def balanced_bounds(work: torch.Tensor, world: int) -> list[tuple[int, int]]:
    """Contiguous shards of (nearly) equal total work.

    ``work``: per-row work estimate (int64, any device, e.g.
    PathSimEngine.row_work()).  Rank r gets the rows whose work prefix falls in
    [r/world, (r+1)/world) of the total.  Every rank computes the same bounds
    from the same C, so no communication is needed.
    """
    n = int(work.numel())
    if world < 1:
        raise ValueError(f"bad world {world}")
    if world == 1 or n == 0:
        return [shard_bounds(n, r, world) for r in range(world)]
    pre = torch.cumsum(work.to(torch.int64), 0)
    total = pre[-1]
    cuts = torch.arange(1, world, device=pre.device, dtype=torch.int64) * total // world
    idx = torch.searchsorted(pre, cuts, right=True).cpu().tolist()
    edges = [0] + [min(max(int(i), 0), n) for i in idx] + [n]
    for i in range(1, len(edges)):
        edges[i] = max(edges[i], edges[i - 1])
    return [(edges[r], edges[r + 1]) for r in range(world)]


def gather_topk(parts, n_rows: int, world: int, group=None, out=None, bounds=None):
    """All-gather every rank's top-k block into the full [n_rows, k] tensors.

    ``parts``: this rank's (idx, cnt, score) tensors with shape [max_shard, k]
    (rows past its shard are padding).  Returns (idx, cnt, score) for all
    n_rows rows in row order on every rank; ``out`` may hold preallocated
    [world * max_shard, k] receive buffers (reused across steps).  ``bounds``:
    the shards in use (default: equal row counts, shard_bounds).
    """
    if bounds is None:
        bounds = [shard_bounds(n_rows, r, world) for r in range(world)]
    if world == 1:
        return tuple(p[:bounds[0][1]] for p in parts)
    m = max_shard(n_rows, world, bounds)
    if out is None:
        out = tuple(torch.empty((world * m,) + tuple(p.shape[1:]), dtype=p.dtype, device=p.device)
                    for p in parts)
    for src, dst in zip(parts, out):
        if src.shape[0] != m:
            raise ValueError(f"part has {src.shape[0]} rows, expected max_shard {m}")
        if dist.get_backend(group) == "nccl":
            dist.all_gather_into_tensor(dst, src.contiguous(), group=group)
        else:   # gloo (CPU tests, one-GPU rehearsal): host staging
            host = dst.cpu() if dst.is_cuda else dst
            dist.all_gather(list(host.view(world, m, *src.shape[1:]).unbind(0)),
                            src.contiguous().cpu(), group=group)
            if host is not dst:
                dst.copy_(host)
    rows = [slice(r * m, r * m + (b - a)) for r, (a, b) in enumerate(bounds)]
    return tuple(torch.cat([o[s] for s in rows]) for o in out)
