"""Row sharding of the all-pairs top-k across ranks.

Every source row's top-k depends only on that row of C plus all of C and g,
so ranks split the author rows into contiguous, work-balanced shards and
exchange nothing but the finished top-k blocks.  One process per GPU; on the
GPU box the collective is RCCL over xGMI called through libdpathsim's C ABI
(:class:`RcclComm`, dps_comm_* / dps_gather -- torch.distributed only carries
the 128-byte unique id at start-up and the barriers), and gloo in the CPU
tests.

Results travel as ONE packed int64 buffer per rank, ``[rows, 2k]``: word 0..k-1
holds (count << 32) | target index, word k..2k-1 the score's fp64 bits (16 B
per entry; counts fit 32 bits because the engine checks max M[x,x] < 2^31 and
M[x,y] <= max(M[x,x], M[y,y])).  They are gathered to rank 0 with a single
``gather`` (not all-gathered to every rank), or written as per-rank shard files
in row order when the result is too large for one host (config 5: 3M x top-100).
"""
from __future__ import annotations

import ctypes as C
import json
import os

import numpy as np
import torch
import torch.distributed as dist


class RcclComm:
    """An RCCL communicator owned by libdpathsim (dps_comm_init: one rank per
    process, on the current device).  Rank 0 creates the unique id
    (dps_comm_get_id); ``group`` -- any torch.distributed group, e.g. gloo --
    only broadcasts those bytes.  Collectives run on the caller's current HIP
    stream (dps_gather / dps_bcast)."""

    def __init__(self, group=None, device=None):
        from . import _lib
        self._lib = _lib
        lib = _lib.load()
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = (torch.device("cuda", torch.cuda.current_device()) if device is None
                       else torch.device(device))
        nb = int(lib.dps_comm_id_bytes())
        buf = (C.c_uint8 * nb)()
        if self.rank == 0:
            _lib.call("dps_comm_get_id", C.addressof(buf))
        cpu = dist.get_backend(group) != "nccl"
        t = torch.tensor(bytearray(buf), dtype=torch.uint8,
                         device="cpu" if cpu else self.device)
        dist.broadcast(t, src=0, group=group)
        buf = (C.c_uint8 * nb)(*t.cpu().tolist())
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            _lib.call("dps_comm_init", C.addressof(h), self.world, self.rank, C.addressof(buf))
        self._h = h

    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def gather(self, send: torch.Tensor, recv: torch.Tensor | None, root: int = 0):
        """Every rank's ``send`` bytes into ``recv`` on ``root`` (rank r at
        byte offset r * send.nbytes); device tensors, current stream."""
        send = send.contiguous()
        nb = send.numel() * send.element_size()
        if self.rank == root:
            if recv is None or recv.numel() * recv.element_size() < self.world * nb:
                raise ValueError("receive buffer smaller than world * send bytes")
        with torch.cuda.device(self.device):
            self._lib.call("dps_gather", self._h, send.data_ptr(),
                           recv.data_ptr() if recv is not None else None, nb, root, self._stream())
        return recv

    def bcast(self, buf: torch.Tensor, root: int = 0):
        with torch.cuda.device(self.device):
            self._lib.call("dps_bcast", self._h, buf.data_ptr(), buf.numel() * buf.element_size(),
                           root, self._stream())
        return buf

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.call("dps_comm_destroy", self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def shard_bounds(n_rows: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous balanced shard [r0, r1) of rank ``rank`` out of ``world``."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    return n_rows * rank // world, n_rows * (rank + 1) // world


def max_shard(n_rows: int, world: int, bounds=None) -> int:
    if bounds is None:
        bounds = [shard_bounds(n_rows, r, world) for r in range(world)]
    return max(b - a for a, b in bounds)


def balanced_edges(work: torch.Tensor, world: int) -> torch.Tensor:
    """Shard edges [0, e_1, ..., n] (int64 tensor on work's device, nothing read
    back): rank r gets the rows whose work prefix falls in [r/world,
    (r+1)/world) of the total.  See :func:`balanced_bounds`."""
    n = int(work.numel())
    if world < 1:
        raise ValueError(f"bad world {world}")
    if world == 1 or n == 0:
        return torch.tensor([shard_bounds(n, r, world)[0] for r in range(world)] + [n],
                            dtype=torch.int64, device=work.device)
    pre = torch.cumsum(work.to(torch.int64), 0)
    cuts = torch.arange(1, world, device=pre.device, dtype=torch.int64) * pre[-1] // world
    idx = torch.searchsorted(pre, cuts, right=True).clamp_(0, n)
    edges = torch.cat([idx.new_zeros(1), idx, idx.new_full((1,), n)])
    return torch.cummax(edges, 0).values


def balanced_bounds(work: torch.Tensor, world: int) -> list[tuple[int, int]]:
    """Contiguous shards of (nearly) equal total work.

    ``work``: per-row work estimate (int64, any device, e.g.
    PathSimEngine.row_work()).  Rank r gets the rows whose work prefix falls in
    [r/world, (r+1)/world) of the total.  Every rank computes the same bounds
    from the same C, so no communication is needed.
    """
    edges = balanced_edges(work, world).cpu().tolist()
    return [(edges[r], edges[r + 1]) for r in range(world)]


# ---------------------------------------------------------------- packing
def pack_topk(idx: torch.Tensor, cnt: torch.Tensor, score: torch.Tensor, out=None):
    """(idx int32, cnt int64, score f64) [R, k] -> int64 [R, 2k] (see module doc)."""
    R, k = idx.shape
    if out is None:
        out = torch.empty((R, 2 * k), dtype=torch.int64, device=idx.device)
    lo = idx.to(torch.int64) & 0xFFFFFFFF
    out[:, :k] = (cnt.to(torch.int64) << 32) | lo
    out[:, k:] = score.contiguous().view(torch.int64)
    return out


def unpack_topk(packed: torch.Tensor):
    """Inverse of :func:`pack_topk`."""
    k = packed.shape[1] // 2
    w = packed[:, :k]
    idx = (w & 0xFFFFFFFF).to(torch.int32)            # -1 round-trips through the low word
    cnt = w >> 32
    score = packed[:, k:].contiguous().view(torch.float64)
    return idx, cnt, score


def gather_topk(parts, n_rows: int, world: int, group=None, out=None, bounds=None, dst: int = 0):
    """Gather every rank's top-k block to rank ``dst`` in ONE collective.

    ``parts``: this rank's (idx, cnt, score) tensors with shape [max_shard, k]
    (rows past its shard are padding) -- or an already packed int64
    [max_shard, 2k] tensor.  Returns (idx, cnt, score) for all n_rows rows in
    row order on rank ``dst`` and None on the other ranks.  ``out``: an optional
    preallocated receive buffer [world * max_shard, 2k] (int64) on ``dst``.
    ``bounds``: the shards in use (default: equal row counts, shard_bounds).
    """
    if bounds is None:
        bounds = [shard_bounds(n_rows, r, world) for r in range(world)]
    packed = parts if isinstance(parts, torch.Tensor) else pack_topk(*parts)
    if world == 1:
        return unpack_topk(packed[:bounds[0][1] - bounds[0][0]])
    m = max_shard(n_rows, world, bounds)
    if packed.shape[0] != m:
        raise ValueError(f"part has {packed.shape[0]} rows, expected max_shard {m}")
    rank = dist.get_rank(group)
    nccl = dist.get_backend(group) == "nccl"
    src = packed.contiguous() if nccl else packed.contiguous().cpu()
    recv = None
    if rank == dst:
        if out is None or not nccl:
            out = torch.empty((world * m, packed.shape[1]), dtype=torch.int64,
                              device=src.device)
        recv = list(out.view(world, m, packed.shape[1]).unbind(0))
    dist.gather(src, gather_list=recv, dst=dst, group=group)
    if rank != dst:
        return None
    rows = [out[r * m: r * m + (b - a)] for r, (a, b) in enumerate(bounds)]
    full = torch.cat(rows)
    if full.device != packed.device:
        full = full.to(packed.device)
    return unpack_topk(full)


# ------------------------------------------------------ compact (8 B) gather
def pack_counts(idx: torch.Tensor, cnt: torch.Tensor, out=None):
    """(idx int32, cnt int64) [R, k] -> int64 [R, k] = (count << 32) | index: the
    score is NOT sent -- the root recomputes it (:func:`rescore`)."""
    if out is None:
        out = torch.empty(idx.shape, dtype=torch.int64, device=idx.device)
    torch.bitwise_or(cnt.to(torch.int64) << 32, idx.to(torch.int64) & 0xFFFFFFFF, out=out)
    return out


def rescore(packed: torch.Tensor, den: torch.Tensor, row_begin: int = 0):
    """(idx, cnt, score) from :func:`pack_counts` words of rows row_begin...:
    score = double(2 cnt) / double(den[x] + den[y]) -- the hot kernel's one fp64
    division of the same exact integers (DPathSim_APVPA.py:51-52), so the bits
    are identical -- and 0.0 for zero counts and empty (-1) slots."""
    idx = (packed & 0xFFFFFFFF).to(torch.int32)
    cnt = packed >> 32
    rows = torch.arange(row_begin, row_begin + packed.shape[0], device=packed.device)
    den = den.to(packed.device)
    y = idx.to(torch.int64).clamp_min(0)
    num = (2 * cnt).to(torch.float64)
    dsum = (den[rows].unsqueeze(1) + den[y]).to(torch.float64)
    score = torch.where((idx >= 0) & (cnt > 0), num / dsum, torch.zeros_like(num))
    return idx, cnt, score


def gather_topk_compact(parts, den: torch.Tensor, n_rows: int, world: int, group=None,
                        out=None, bounds=None, dst: int = 0, force_collective: bool = False,
                        comm: RcclComm | None = None):
    """As :func:`gather_topk`, with 8 B per slot on the wire: every rank sends
    (count << 32) | index words; rank ``dst`` rebuilds the scores from its own
    copy of the denominator term ``den`` (every rank holds all of g).  ``parts``:
    (idx, cnt[, score]) [max_shard, k] or packed int64 [max_shard, k].
    ``comm``: gather with libdpathsim's RCCL communicator (dps_gather) instead
    of torch.distributed.  ``force_collective`` runs the gather even for one
    rank (lets a one-GPU box exercise the RCCL call)."""
    if bounds is None:
        bounds = [shard_bounds(n_rows, r, world) for r in range(world)]
    packed = parts if isinstance(parts, torch.Tensor) else pack_counts(parts[0], parts[1])
    if world == 1 and not force_collective:
        return rescore(packed[:bounds[0][1] - bounds[0][0]], den)
    m = max_shard(n_rows, world, bounds)
    if packed.shape[0] != m:
        raise ValueError(f"part has {packed.shape[0]} rows, expected max_shard {m}")
    if comm is not None:
        if comm.rank == dst and (out is None or out.numel() < world * m * packed.shape[1]):
            out = torch.empty((world * m, packed.shape[1]), dtype=torch.int64, device=packed.device)
        comm.gather(packed, out if comm.rank == dst else None, root=dst)
        if comm.rank != dst:
            return None
        full = torch.cat([out[r * m: r * m + (b - a)] for r, (a, b) in enumerate(bounds)])
        return rescore(full, den)
    rank = dist.get_rank(group)
    nccl = dist.get_backend(group) == "nccl"
    src = packed.contiguous() if nccl else packed.contiguous().cpu()
    recv = None
    if rank == dst:
        if out is None or not nccl:
            out = torch.empty((world * m, packed.shape[1]), dtype=torch.int64, device=src.device)
        recv = list(out.view(world, m, packed.shape[1]).unbind(0))
    dist.gather(src, gather_list=recv, dst=dst, group=group)
    if rank != dst:
        return None
    full = torch.cat([out[r * m: r * m + (b - a)] for r, (a, b) in enumerate(bounds)])
    return rescore(full.to(packed.device), den)


# ------------------------------------------------------- per-rank shard files
def write_topk_shard(directory, rank: int, world: int, bounds, parts, k: int) -> str:
    """Write this rank's rows [r0, r1) as ``topk_rank{rank:05d}.npy`` (packed int64
    [r1-r0, 2k]) plus a JSON manifest entry -- the per-rank output the survey
    asks for when one gathered result would not fit a host."""
    os.makedirs(directory, exist_ok=True)
    r0, r1 = bounds[rank]
    packed = parts if isinstance(parts, torch.Tensor) else pack_topk(*parts)
    arr = packed[: r1 - r0].cpu().numpy()
    path = os.path.join(directory, f"topk_rank{rank:05d}.npy")
    np.save(path, arr, allow_pickle=False)
    with open(os.path.join(directory, f"topk_rank{rank:05d}.json"), "w") as f:
        json.dump({"rank": rank, "world": world, "row_begin": r0, "row_end": r1, "k": k,
                   "layout": "int64 [rows, 2k]: (cnt << 32) | idx, then f64 score bits"}, f)
    return path


def read_topk_shards(directory):
    """Merge the shard files of :func:`write_topk_shard` in row order (host tensors)."""
    metas = []
    for name in sorted(os.listdir(directory)):
        if name.startswith("topk_rank") and name.endswith(".json"):
            with open(os.path.join(directory, name)) as f:
                metas.append(json.load(f))
    if not metas:
        raise FileNotFoundError(f"no topk shards in {directory}")
    metas.sort(key=lambda m: m["row_begin"])
    world = metas[0]["world"]
    if len(metas) != world or any(m["world"] != world for m in metas):
        raise ValueError(f"{len(metas)} shard files for world {world}")
    if metas[0]["row_begin"] != 0:
        raise ValueError("the first shard does not start at row 0")
    k = metas[0]["k"]
    if any(m["k"] != k for m in metas):
        raise ValueError("shards disagree on k")
    for a, b in zip(metas, metas[1:]):
        if a["row_end"] != b["row_begin"]:
            raise ValueError("shards do not tile the rows")
    blocks = []
    for m in metas:
        arr = np.load(os.path.join(directory, f"topk_rank{m['rank']:05d}.npy"), allow_pickle=False)
        if arr.shape != (m["row_end"] - m["row_begin"], 2 * k) or arr.dtype != np.int64:
            raise ValueError(f"shard of rank {m['rank']} has shape {arr.shape} {arr.dtype}, "
                             f"manifest says {m['row_end'] - m['row_begin']} x {2 * k} int64")
        blocks.append(arr)
    return unpack_topk(torch.from_numpy(np.concatenate(blocks)))
