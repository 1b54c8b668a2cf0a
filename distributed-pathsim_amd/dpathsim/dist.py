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
        err = ""
        if self.rank == 0:
            try:
                _lib.call("dps_comm_get_id", C.addressof(buf))
            except RuntimeError as e:   # broadcast the failure too: no rank waits forever
                err = str(e)
        cpu = dist.get_backend(group) != "nccl"
        t = torch.tensor(bytearray(buf) + bytes([0 if err else 1]), dtype=torch.uint8,
                         device="cpu" if cpu else self.device)
        # src is a GLOBAL rank: the group's rank 0 (a subgroup need not hold rank 0)
        src = 0 if group is None else dist.get_global_rank(group, 0)
        dist.broadcast(t, src=src, group=group)
        b = t.cpu().tolist()
        if b[nb] != 1:
            raise RuntimeError(f"dps_comm_get_id failed on rank 0 {err}".rstrip())
        buf = (C.c_uint8 * nb)(*b[:nb])
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

    def allgather(self, send: torch.Tensor, recv: torch.Tensor):
        """Every rank's ``send`` bytes into ``recv`` on every rank (rank r at
        byte offset r * send.nbytes); device tensors, current stream."""
        send = send.contiguous()
        nb = send.numel() * send.element_size()
        if recv.numel() * recv.element_size() < self.world * nb:
            raise ValueError("receive buffer smaller than world * send bytes")
        with torch.cuda.device(self.device):
            self._lib.call("dps_allgather", self._h, send.data_ptr(), recv.data_ptr(), nb,
                           self._stream())
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


def check_comm_gather(comm, device, group=None, n: int = 4099) -> bool:
    """One gather of a known pattern through ``comm`` (anything with
    ``rank``/``world``/``gather(send, recv, root)``, e.g. :class:`RcclComm`),
    checked by rank 0 in this process; the verdict is shared over ``group``
    (the control-plane group: gloo in bench.py) so every rank returns the same
    answer.  A gather that raises counts as a mismatch.  bench.py runs it once
    before its timed loop and, on a mismatch, takes the torch nccl group for
    the top-k gather instead."""
    device = torch.device(device)
    ok = True
    try:
        ar = torch.arange(n, dtype=torch.int64, device=device)
        send = ar * 1000003 + comm.rank * 7919 + 1
        recv = (torch.full((comm.world * n,), -1, dtype=torch.int64, device=device)
                if comm.rank == 0 else None)
        comm.gather(send, recv, root=0)
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        if comm.rank == 0:
            want = torch.cat([ar * 1000003 + r * 7919 + 1 for r in range(comm.world)])
            ok = bool(torch.equal(recv, want))
    except Exception:       # noqa: BLE001 -- any failure means: do not use this path
        ok = False
    nccl = dist.get_backend(group) == "nccl"
    verdict = torch.tensor([1 if ok else 0], dtype=torch.int64,
                           device=device if nccl else "cpu")
    dist.all_reduce(verdict, op=dist.ReduceOp.MIN, group=group)
    return int(verdict.item()) == 1


class TileSplit:
    """The N > 1 build's tile split (PathSimEngine.split): rank r builds the C^T
    tiles of its own target-tile range (dps_label_rows + dps_ct_tiles_build2
    over that sub-C), the ranks all-gather the slices, and every rank assembles
    the full layout (dps_tiles_assemble).  ``allgather(send, recv)`` is a
    collective on the current stream (RCCL through :class:`RcclComm` or the
    nccl process group; over gloo the bytes go through host memory), and
    ``allreduce_max(int)`` a host-value collective for the plan.  ``caps`` --
    tile width -> slice entry capacity -- is the plan every later build of the
    same graph gathers with (PathSimEngine.check sets it after the first)."""

    def __init__(self, rank: int, world: int, allgather, allreduce_max):
        if world < 1 or not 0 <= rank < world:
            raise ValueError(f"bad rank {rank} / world {world}")
        self.rank, self.world = rank, world
        self.allgather = allgather
        self.allreduce_max = allreduce_max
        self.caps = {}

    @classmethod
    def from_group(cls, group=None, comm: "RcclComm | None" = None, device=None):
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        nccl = dist.get_backend(group) == "nccl"
        dev = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())

        if comm is not None:
            def ag(send, recv):
                comm.allgather(send, recv)
        elif nccl:
            def ag(send, recv):
                dist.all_gather_into_tensor(recv, send, group=group)
        else:
            def ag(send, recv):          # gloo (CPU rehearsals): through host memory
                parts = [torch.empty_like(send, device="cpu") for _ in range(world)]
                dist.all_gather(parts, send.cpu(), group=group)
                recv.copy_(torch.cat(parts).to(recv.device))

        def amax(v: int) -> int:
            t = torch.tensor([int(v)], dtype=torch.int64, device=dev if nccl else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
            return int(t.item())

        return cls(rank, world, ag, amax)


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


def _stream(t: torch.Tensor):
    return torch.cuda.current_stream(t.device).cuda_stream


def shard_edges(terms: torch.Tensor, world: int, out: torch.Tensor | None = None,
                ref: torch.Tensor | None = None, mismatch: torch.Tensor | None = None):
    """Shard edges from the build's per-row work terms (``row_terms``): the same
    plan as ``balanced_edges(terms + (terms.sum() // n) // 2, world)``
    (PathSimEngine.row_work), computed by dps_shard_edges on the device for a
    device tensor -- one scan and a binary search per cut, nothing read back,
    no PyTorch compute.  ``ref`` / ``mismatch``: add the number of edges that
    differ from ``ref`` to the int64 device scalar ``mismatch`` (the timed
    step's plan check).  Host tensors (the CPU gloo tests) take the same
    arithmetic in PyTorch."""
    n = int(terms.numel())
    if not terms.is_cuda:
        w = terms.to(torch.int64)
        hm = (w.sum() // max(n, 1)) // 2 if n else 0
        e = balanced_edges(w + hm, world) if world > 1 and n else \
            torch.tensor([shard_bounds(n, r, world)[0] for r in range(world)] + [n], dtype=torch.int64)
        if out is not None:
            out.copy_(e)
        if ref is not None:
            mismatch.add_((e != ref.to(e.device)).sum().to(mismatch.device))
        return e if out is None else out
    from . import _lib
    terms = terms.contiguous()
    if terms.dtype != torch.int64:
        raise TypeError("terms must be int64")
    if out is None:
        out = torch.empty(world + 1, dtype=torch.int64, device=terms.device)
    if ref is not None and mismatch is None:
        raise ValueError("ref needs a mismatch counter")
    ws = torch.empty(max(_lib.size("dps_shard_edges_workspace_size", n), 256), dtype=torch.uint8,
                     device=terms.device)
    _lib.call("dps_shard_edges", terms.data_ptr(), n, world, out.data_ptr(),
              ref.data_ptr() if ref is not None else None,
              mismatch.data_ptr() if mismatch is not None else None, ws.data_ptr(), ws.numel(),
              _stream(terms))
    return out


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
        if not nccl or not _recv_ok(out, world * m, int(packed.shape[1]), src.device):
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
    score is NOT sent -- the root recomputes it (:func:`rescore`).  Device
    tensors: dps_pack_counts (HIP); host tensors: the same in PyTorch."""
    if out is None:
        out = torch.empty(idx.shape, dtype=torch.int64, device=idx.device)
    if idx.is_cuda:
        from . import _lib
        if not (idx.is_contiguous() and cnt.is_contiguous() and out.is_contiguous()
                and idx.dtype == torch.int32 and cnt.dtype == torch.int64
                and out.dtype == torch.int64 and idx.shape == cnt.shape
                and out.numel() >= idx.numel()):
            raise ValueError("pack_counts: contiguous int32 idx / int64 cnt / int64 out of one shape")
        _lib.call("dps_pack_counts", idx.data_ptr(), cnt.data_ptr(), idx.numel(), out.data_ptr(),
                  _stream(idx))
        return out
    torch.bitwise_or(cnt.to(torch.int64) << 32, idx.to(torch.int64) & 0xFFFFFFFF, out=out)
    return out


def unpack_gathered(gathered: torch.Tensor, world: int, m: int, edges: torch.Tensor,
                    den: torch.Tensor, out=None):
    """Rank 0's gathered [world * m, k] words -> (idx, cnt, score) of rows
    [edges[0], edges[world]) in row order (dps_unpack_gathered, HIP): rank r's
    rows are gathered rows r*m ..; the score is the kernel's division of the
    same exact integers, bit-identical.  ``edges``: int64 device [world + 1];
    its host copy gives the row count (pass ``out`` to skip that read)."""
    from . import _lib
    k = int(gathered.shape[1])
    if out is None:
        e = edges.cpu()
        n = int(e[world] - e[0])
        out = (torch.empty((n, k), dtype=torch.int32, device=gathered.device),
               torch.empty((n, k), dtype=torch.int64, device=gathered.device),
               torch.empty((n, k), dtype=torch.float64, device=gathered.device))
    idx, cnt, sc = out
    n = int(idx.shape[0])
    for t, dt in ((idx, torch.int32), (cnt, torch.int64), (sc, torch.float64)):
        if not (t.is_contiguous() and t.dtype == dt and tuple(t.shape) == (n, k)
                and t.device == gathered.device):
            raise ValueError("unpack_gathered: outputs must be contiguous [n, k] int32 / int64 / f64 "
                             "on the gathered tensor's device")
    if not (gathered.is_contiguous() and gathered.dtype == torch.int64 and edges.is_cuda
            and edges.dtype == torch.int64 and edges.numel() == world + 1
            and gathered.shape[0] >= world * m):
        raise ValueError("unpack_gathered: int64 gathered [>= world*m, k] and int64 device edges [world+1]")
    den = den.contiguous()
    _lib.call("dps_unpack_gathered", gathered.data_ptr(), world, m, k, edges.data_ptr(), n,
              den.data_ptr(), idx.data_ptr(), cnt.data_ptr(), sc.data_ptr(), _stream(gathered))
    return idx, cnt, sc


def rescore(packed: torch.Tensor, den: torch.Tensor, row_begin: int = 0):
    """(idx, cnt, score) from :func:`pack_counts` words of rows row_begin...:
    score = double(2 cnt) / double(den[x] + den[y]) -- the hot kernel's one fp64
    division of the same exact integers (DPathSim_APVPA.py:51-52), so the bits
    are identical -- and 0.0 for zero counts and empty (-1) slots.  Device
    tensors: dps_unpack_gathered (HIP); host tensors: the same in PyTorch."""
    if packed.is_cuda:
        R = int(packed.shape[0])
        edges = torch.tensor([row_begin, row_begin + R], dtype=torch.int64, device=packed.device)
        k = int(packed.shape[1])
        out = (torch.empty((R, k), dtype=torch.int32, device=packed.device),
               torch.empty((R, k), dtype=torch.int64, device=packed.device),
               torch.empty((R, k), dtype=torch.float64, device=packed.device))
        return unpack_gathered(packed.contiguous(), 1, R, edges, den.to(packed.device), out=out)
    idx = (packed & 0xFFFFFFFF).to(torch.int32)
    cnt = packed >> 32
    rows = torch.arange(row_begin, row_begin + packed.shape[0], device=packed.device)
    den = den.to(packed.device)
    y = idx.to(torch.int64).clamp_min(0)
    num = (2 * cnt).to(torch.float64)
    dsum = (den[rows].unsqueeze(1) + den[y]).to(torch.float64)
    score = torch.where((idx >= 0) & (cnt > 0), num / dsum, torch.zeros_like(num))
    return idx, cnt, score


def _recv_ok(out, rows, cols, device) -> bool:
    """A caller-supplied receive buffer is used only if it is exactly what the
    collective writes: contiguous int64 [rows, cols] on ``device``."""
    return (out is not None and out.is_contiguous() and out.dtype == torch.int64
            and tuple(out.shape) == (rows, cols) and out.device == device)


def gather_topk_compact(parts, den: torch.Tensor, n_rows: int, world: int, group=None,
                        out=None, bounds=None, dst: int = 0, force_collective: bool = False,
                        comm: RcclComm | None = None, edges: torch.Tensor | None = None,
                        result=None):
    """As :func:`gather_topk`, with 8 B per slot on the wire: every rank sends
    (count << 32) | index words; rank ``dst`` rebuilds the scores from its own
    copy of the denominator term ``den`` (every rank holds all of g).  ``parts``:
    (idx, cnt[, score]) [max_shard, k] or packed int64 [max_shard, k].
    ``comm``: gather with libdpathsim's RCCL communicator (dps_gather) instead
    of torch.distributed.  ``force_collective`` runs the gather even for one
    rank (lets a one-GPU box exercise the RCCL call).  On the device the
    rows are put back in order and rescored by one HIP kernel
    (dps_unpack_gathered) reading the gathered buffer in place; ``edges`` (int64
    device [world + 1], the shard edges) and ``result`` ((idx, cnt, score)
    [n_rows, k]) avoid building them from ``bounds`` inside a timed step."""
    if bounds is None:
        bounds = [shard_bounds(n_rows, r, world) for r in range(world)]
    packed = parts if isinstance(parts, torch.Tensor) else pack_counts(parts[0], parts[1])
    if world == 1 and not force_collective:
        return rescore(packed[:bounds[0][1] - bounds[0][0]], den)
    m = max_shard(n_rows, world, bounds)
    if packed.shape[0] != m:
        raise ValueError(f"part has {packed.shape[0]} rows, expected max_shard {m}")
    cols = int(packed.shape[1])

    def finish(buf):
        if buf.is_cuda:
            e = edges if edges is not None else torch.tensor(
                [a for a, _ in bounds] + [bounds[-1][1]], dtype=torch.int64, device=buf.device)
            return unpack_gathered(buf, world, m, e, den.to(buf.device), out=result)
        full = torch.cat([buf[r * m: r * m + (b - a)] for r, (a, b) in enumerate(bounds)])
        return rescore(full, den.to(full.device))

    if comm is not None:
        if comm.rank == dst and not _recv_ok(out, world * m, cols, packed.device):
            out = torch.empty((world * m, cols), dtype=torch.int64, device=packed.device)
        comm.gather(packed, out if comm.rank == dst else None, root=dst)
        if comm.rank != dst:
            return None
        return finish(out)
    rank = dist.get_rank(group)
    nccl = dist.get_backend(group) == "nccl"
    src = packed.contiguous() if nccl else packed.contiguous().cpu()
    recv = None
    if rank == dst:
        if not nccl or not _recv_ok(out, world * m, cols, src.device):
            out = torch.empty((world * m, cols), dtype=torch.int64, device=src.device)
        recv = list(out.view(world, m, cols).unbind(0))
    dist.gather(src, gather_list=recv, dst=dst, group=group)
    if rank != dst:
        return None
    return finish(out.to(packed.device))


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
