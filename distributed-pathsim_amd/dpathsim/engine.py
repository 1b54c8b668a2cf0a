"""Device pipeline: typed CSR build -> SpGEMM C -> s, g -> C^T tiles -> top-k.

Every stage is a libdpathsim (HIP, gfx950) call on the current PyTorch-ROCm
stream; PyTorch only allocates device memory.  Replaces the graphframes motif
queries of DPathSim_APVPA.py:70-109 (see include/dpathsim.h per entry point).
"""
from __future__ import annotations

import ctypes as C
import math
import os
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from ._lib import DPS_ERR_OVERFLOW
from .graph import TypedTables

# one tile of 16384 targets per wave: 4-bit counters in 8 KiB of LDS (a tile
# whose bound exceeds 15 runs as two u8 halves); 8192 = u8 counters.  None =
# by shape (auto_tile_w): the 4-bit tiles pay when a typical row's bound
# sum_v C[x,v] fits 4 bits -- config3: 7.5 per author, 80.3 -> 75.3 ms per
# step; config4 (APTPA, ~30 topic papers per author): 224.9 ms at 16384
# against 205.3 at 8192 (profiles/r03/c45)
DEFAULT_TILE_W = None
AUTO_TILE_W_MAX_ROW_SUM = 15.0
DEFAULT_SPLIT_ROWS = 256    # heaviest rows of a launch cut into pieces
DEFAULT_PIECES = 16         # target-tile ranges per split row
DEFAULT_HEAVY_VENUES = 32   # venue skipping: heavy venues in the dense table (64-byte rows)
# venue skipping is exact; on config3 it scatters 41 % fewer chunks: at tile_w
# 16384 the hot kernel takes 74.1 against 77.9 ms (profiles/r03/d), at 8192
# 89.4 against 86.9 ms (profiles/r03/a) -- on by default for 16384 only
VENUE_SKIP_TILE_W = (16384, 15360)
SYM_TILE_W = (8192, 16384)
# the T15 layout (dps_cct1.hip Geo, round 6): 15 / 16 of 8192 / 16384 targets per
# tile, so a wave's accumulator is 7680 bytes and 20 one-wave workgroups stay
# resident per CU (8 KiB keeps 18: the CU's LDS is ~150 KiB in 512-byte granules)
T15_TILE_W = (7680, 15360)
FOUR_BIT_TILE_W = (16384, 15360)   # 4-bit counters, companion u8 halves at tile_w / 2


def valid_tile_w(w: int) -> bool:
    return w in T15_TILE_W or (not w & (w - 1) and 256 <= w <= 65536)
DEFAULT_SYM_BAND = 1          # tiles either side of a row's own scanned by both rows
DEFAULT_SYM_REC_PER_ROW = 32  # record capacity per row (config3: about 5 per row needed)


def _ptr(t):
    return None if t is None else t.data_ptr()


@dataclass
class BuildInfo:
    n_nodes: int = 0
    n_edges: int = 0
    n_authors: int = 0
    n_papers: int = 0
    n_mids: int = 0
    nnz_ap: int = 0
    nnz_px: int = 0
    expand: int = 0
    nnz_c: int = 0
    max_c: int = 0
    max_diag: int = 0
    max_g: int = 0
    phase_ms: dict = field(default_factory=dict)


@dataclass
class Bounds:
    """Host-side capacity bounds, computed once from the raw (not yet distinct)
    typed edge list at upload, so that build() never reads a size back from the
    device: every count after distinct() is at most its raw-edge count."""
    expand: int = 1      # >= sum_{x author} sum_{p in AP[x]} |PX[p]| (SpGEMM expansion)
    sum_c: int = 1       # >= sum of C over all AP rows (>= sum of s)
    key_bits: int = 1    # >= bit length of max g (and of max M[x,x])
    max_row_expand: int = 1   # >= max over AP rows of sum_{p in AP[row]} |PX[p]|
    max_mids_per_paper: int = 0   # >= max |PX[p]| (raw edges, before distinct)


DENOMINATORS = ("rowsum", "diag")


class PathSimEngine:
    """All device state for one graph + meta-path on one GPU.

    ``denominator``: ``'rowsum'`` (default) is the reference's global walk
    g[x] = sum_y M[x,y] (DPathSim_APVPA.py:70-88); ``'diag'`` is the
    textbook PathSim M[x,x] + M[y,y].  It only changes which per-author term the
    top-k kernel adds in the score's denominator.
    """

    def __init__(self, typed: TypedTables, device=None, tile_w: int | None = DEFAULT_TILE_W,
                 denominator: str = "rowsum"):
        if not torch.cuda.is_available():
            raise RuntimeError("PathSimEngine needs a ROCm GPU (torch.cuda.is_available() is False);"
                               " there is no CPU fallback")
        _lib.load()
        self.typed = typed
        self.device = torch.device(device if device is not None else "cuda")
        self.bounds = None
        if tile_w is None:
            self.bounds = host_bounds(typed)
            tile_w = auto_tile_w(typed, self.bounds)
        if not valid_tile_w(int(tile_w)):
            raise ValueError("tile_w must be a power of two in [256, 65536], 7680 or 15360")
        if denominator not in DENOMINATORS:
            raise ValueError(f"denominator must be one of {DENOMINATORS}")
        self.tile_w = int(tile_w)
        self.denominator = denominator
        self.tile_skip = True
        # multi-mid SpGEMM: "sort" (expand + segmented sort/unique) or "hash"
        self.spgemm = "sort"
        # venue skipping (dps_venue_skip): exact, row-sum denominator only
        self.venue_skip = tile_w in VENUE_SKIP_TILE_W and denominator == "rowsum"
        self.n_heavy = DEFAULT_HEAVY_VENUES
        # 4-bit tiles (16384 / 15360): the companion u8 tiles of half the width
        self.half_tiles = True
        # ... built together with the 4-bit tiles in one walk of C (round 6)
        self.dual_build = True
        # ... and optimistic 4-bit passes over tiles whose bound is 16..255
        # (dps_cct_ext.tile_sum; exact either way, fewer passes)
        self.opt_passes = False   # round 4: measured, see DESIGN §6 (off until it wins)
        self._ext = None
        # symmetric mode (dps_cct_sym): every pair scanned once; whole-range
        # launches at tile_w 8192 / 16384 (venue skipping does not apply there)
        self.sym = False
        self.sym_band = DEFAULT_SYM_BAND
        self.sym_rec_per_row = DEFAULT_SYM_REC_PER_ROW
        self.defer_checks = False
        self._sym_stat = None
        # load balance of the hot kernel: the split_rows heaviest rows of a
        # launch are cut into `pieces` target-tile ranges (see topk())
        self.split_rows = DEFAULT_SPLIT_ROWS
        self.pieces = DEFAULT_PIECES
        # N > 1 (dist.TileSplit): this rank builds the C^T tiles of its own
        # target-tile range only and the ranks all-gather the slices
        self.split = None
        self.info = BuildInfo()
        self.built = False
        self.checked = False
        self._dev = {}
        self._piece_cache = {}
        self._last_dq = None       # the last top-k launch's dequeue list

    # ------------------------------------------------------------------ utils
    @property
    def stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def _empty(self, n, dtype):
        return torch.empty(max(int(n), 1), dtype=dtype, device=self.device)

    def _ws(self, nbytes):
        return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=self.device)

    # ----------------------------------------------------------------- upload
    def upload(self):
        """Host -> HBM copy of the typed node tables and the raw edge list, plus
        the host-side capacity bounds (:class:`Bounds`)."""
        t = self.typed
        g = t.graph
        with torch.cuda.device(self.device):
            to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(self.device, non_blocking=False)
            self._dev.update(
                edge_src=to(g.edge_src if g.n_edges else np.zeros(1, np.int32)),
                edge_dst=to(g.edge_dst if g.n_edges else np.zeros(1, np.int32)),
                edge_rel=to(t.edge_rel if g.n_edges else np.zeros(1, np.uint8)),
                node_type=to(t.node_type if g.n_nodes else np.zeros(1, np.uint8)),
                node_rowid=to(t.node_rowid if g.n_nodes else np.zeros(1, np.int32)),
                node_colid=to(t.node_colid if g.n_nodes else np.zeros(1, np.int32)),
                # the SpGEMM status of the gather and sort paths, which never
                # write it: zeroed once here, so a build launches no fill for it
                sp_zero=to(np.zeros(1, np.int32)),
            )
        if self.bounds is None:
            self.bounds = host_bounds(t)
        return self

    # ------------------------------------------------------------------ build
    def build(self, timed: bool = False, check: bool = True):
        """Run the device build.  Inputs must be uploaded (resident in HBM).

        Nothing is read back while the work is enqueued: buffers are sized from
        :class:`Bounds`.  The overflow conditions (max C, max M[x,x], max g) are
        checked by :meth:`check` -- here when ``check`` (one synchronisation at
        the end), else by the caller before it trusts the results."""
        if "edge_src" not in self._dev:
            self.upload()
        t = self.typed
        d = self._dev
        st = self.stream
        bnd = self.bounds
        N, E = t.graph.n_nodes, t.graph.n_edges
        NR = t.n_rows             # C row space: authors, other AP sources, one empty row
        NA, NP, NV = t.n_authors, t.n_papers, t.n_mids
        info = self.info = BuildInfo(n_nodes=N, n_edges=E, n_authors=NA, n_papers=NP, n_mids=NV)
        self.checked = False
        marks = []

        def mark(name):
            if timed:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
                marks.append((name, ev))

        with torch.cuda.device(self.device):
            mark("start")
            # A2: typed incidence extraction
            ap_r, ap_c = self._empty(E, torch.int32), self._empty(E, torch.int32)
            px_r, px_c = self._empty(E, torch.int32), self._empty(E, torch.int32)
            n_ap = self._empty(1, torch.int64)
            n_px = self._empty(1, torch.int64)
            _lib.call("dps_extract_incidence", _ptr(d["edge_src"]), _ptr(d["edge_dst"]),
                      _ptr(d["edge_rel"]), E, _ptr(d["node_type"]), _ptr(d["node_rowid"]),
                      _ptr(d["node_colid"]), N, _ptr(ap_r), _ptr(ap_c), _ptr(n_ap),
                      _ptr(px_r), _ptr(px_c), _ptr(n_px), st)
            mark("extract")
            # A2/A3: typed CSR build (distinct)
            ws_bytes = max(_lib.size("dps_csr_build_workspace_size", E, NR),
                           _lib.size("dps_csr_build_workspace_size", E, NP))
            ws = self._ws(ws_bytes)
            ap_ptr, ap_col = self._empty(NR + 1, torch.int64), self._empty(E, torch.int32)
            ap_nnz = self._empty(1, torch.int64)
            _lib.call("dps_csr_build", _ptr(ap_r), _ptr(ap_c), E, _ptr(n_ap), NR, _ptr(ap_ptr),
                      _ptr(ap_col), _ptr(ap_nnz), _ptr(ws), ws.numel(), st)
            single = bnd.max_mids_per_paper <= 1
            if single:
                # at most one raw PX edge per paper: the PX pairs are already
                # distinct -- a paper -> mid map replaces the PX CSR
                vp = self._empty(NP, torch.int32)
                _lib.call("dps_paper_mid_map", _ptr(px_r), _ptr(px_c), E, _ptr(n_px), NP, _ptr(vp),
                          st)
                px_ptr = px_col = None
                px_nnz = n_px
            else:
                px_ptr, px_col = self._empty(NP + 1, torch.int64), self._empty(E, torch.int32)
                px_nnz = self._empty(1, torch.int64)
                _lib.call("dps_csr_build", _ptr(px_r), _ptr(px_c), E, _ptr(n_px), NP, _ptr(px_ptr),
                          _ptr(px_col), _ptr(px_nnz), _ptr(ws), ws.numel(), st)
            del ap_r, ap_c, px_r, px_c
            mark("csr")
            # A3: SpGEMM C = W_AP . W_PX over EVERY AP row (author rows [0, NA)
            # first, then untyped author_of sources), capacities from the
            # raw-edge bounds (sum_c >= nnz C), no size read-back.  Papers with
            # at most one mid (APVPA): gather + segmented unique; otherwise
            # expand + segmented sort/unique (config4: 3.2 ms against 9.8 ms for
            # the hash SpGEMM, kept as engine.spgemm = "hash").
            cap = bnd.sum_c
            c_ptr, c_nnz = self._empty(NR + 1, torch.int64), self._empty(2, torch.int64)
            # (the hash SpGEMM zeroes and sets its own status; the other two
            # paths have none -- their status is the never-written zero word)
            sp_status = d["sp_zero"] if (single or self.spgemm != "hash") else self._empty(1, torch.int32)
            c_col, c_val = self._empty(cap, torch.int32), self._empty(cap, torch.int32)
            if single:
                sws = self._ws(_lib.size("dps_spgemm_single_workspace_size", NR, E, NP))
                for numeric in (False, True):
                    _lib.call("dps_spgemm_single_map", _ptr(ap_ptr), _ptr(ap_col), NR, E, _ptr(vp),
                              None, None, NP, NV, _ptr(c_ptr), _ptr(c_col) if numeric else None,
                              _ptr(c_val) if numeric else None, _ptr(c_nnz), _ptr(sws),
                              sws.numel(), st)
                del vp
            elif self.spgemm != "hash":
                # expand + segmented sort/unique (sum_c bounds the expansion)
                sws = self._ws(_lib.size("dps_spgemm_workspace_size", NR, bnd.sum_c))
                for numeric in (False, True):
                    _lib.call("dps_spgemm_count", _ptr(ap_ptr), _ptr(ap_col), None, NR, _ptr(px_ptr),
                              _ptr(px_col), NP, _ptr(c_ptr), _ptr(c_col) if numeric else None,
                              _ptr(c_val) if numeric else None, _ptr(c_nnz), bnd.sum_c, _ptr(sws),
                              sws.numel(), st)
            else:
                sws = self._ws(_lib.size("dps_spgemm_hash_workspace_size", NR, bnd.max_row_expand))
                for numeric in (False, True):
                    _lib.call("dps_spgemm_hash", _ptr(ap_ptr), _ptr(ap_col), None, NR, _ptr(px_ptr),
                              _ptr(px_col), bnd.max_row_expand, _ptr(c_ptr),
                              _ptr(c_col) if numeric else None, _ptr(c_val) if numeric else None,
                              _ptr(c_nnz), _ptr(sp_status), _ptr(sws), sws.numel(), st)
            del sws
            mark("spgemm")
            # A4: s = column sums of C over ALL AP rows, g = C.s over author rows,
            # diag, stats
            # ... and, in the same two passes over C, the hot kernel's row work
            s = self._empty(NV, torch.int64)
            n_v = self._empty(NV, torch.int32)
            g = self._empty(NA, torch.int64)
            diag = self._empty(NA, torch.int64)
            terms = self._empty(NA, torch.int64)
            stats = self._empty(_lib.STATS_LEN, torch.int64)
            wws = self._ws(_lib.size("dps_walks_workspace_size", cap, NV))
            _lib.call("dps_walks_fused_ws", _ptr(c_ptr), _ptr(c_col), _ptr(c_val), NR, NA, NV,
                      _ptr(s), _ptr(n_v), _ptr(g), _ptr(diag), _ptr(terms), _ptr(stats), cap,
                      _ptr(wws), wws.numel(), st)
            del wws
            mark("walks")
            # the per-author denominator term of the score
            den = g if self.denominator == "rowsum" else diag
            # A5 operand layout: targets relabeled by ascending denominator term,
            # then tiled C^T
            t_perm, t_rank = self._empty(NA, torch.int32), self._empty(NA, torch.int32)
            g_t = self._empty(NA, torch.int64)
            ows = self._ws(_lib.size("dps_target_order_workspace_size", NA))
            _lib.call("dps_target_order", _ptr(den), NA, bnd.key_bits, _ptr(t_perm),
                      _ptr(t_rank), _ptr(g_t), _ptr(ows), ows.numel(), st)
            del ows
            mark("order")
            # (no authors: nothing to split, every rank builds the empty tiles)
            split = (self.split if self.split is not None and self.split.world > 1 and NA > 0
                     else None)
            T = max(1, math.ceil(NA / self.tile_w)) if NA else 1
            ent_cap = _lib.size("dps_ct_tiles_ent_capacity", bnd.expand, bnd.sum_c, NV, NA,
                                self.tile_w)
            if ent_cap >= 2 ** 32:
                raise OverflowError("padded nnz(C) >= 2^32 exceeds the uint32 tile offsets")
            sub = self._label_rows(split, c_ptr, c_col, c_val, t_perm) if split else None
            # the 4-bit tiles and their companion u8 halves from one walk of C
            # (dps_ct_tiles_build_dual) -- replicated builds only
            dual = (not split and self.dual_build and self.half_tiles
                    and self.tile_w in FOUR_BIT_TILE_W)
            half = None
            if split:
                tile_off, tile_ent, tile_maxc, tile_gmin, status = self._split_tiles(
                    split, sub, self.tile_w, g_t, True, ent_cap)
            elif dual:
                hv_slot, hv_c, nh = self._heavy_venues(n_v, NA, NV, st)
                HW = self.tile_w // 2
                T8 = max(1, math.ceil(NA / HW)) if NA else 1
                h_cap = _lib.size("dps_ct_tiles_ent_capacity", bnd.expand, bnd.sum_c, NV, NA, HW)
                tile_off = self._empty(NV * T + 1, torch.int32)
                tile_maxc = self._empty(NV * T + 1, torch.int32)
                tile_gmin = self._empty(T, torch.int64)
                tile_ent = self._empty(ent_cap, torch.int32)
                status = self._empty(1, torch.int32)
                h_off = self._empty(NV * T8 + 1, torch.int32)
                h_maxc = self._empty(NV * T8 + 1, torch.int32)
                h_ent = self._empty(h_cap, torch.int32)
                h_status = self._empty(1, torch.int32)
                tws = self._ws(_lib.size("dps_ct_tiles_workspace_size_dual", NV, NA, self.tile_w,
                                         bnd.expand))
                _lib.call("dps_ct_tiles_build_dual", _ptr(c_ptr), _ptr(c_col), _ptr(c_val),
                          _ptr(den), _ptr(t_rank), NA, NV, self.tile_w, bnd.expand, _ptr(tile_off),
                          _ptr(tile_ent), tile_ent.numel(), _ptr(tile_maxc), _ptr(tile_gmin),
                          _ptr(h_off), _ptr(h_ent), h_ent.numel(), _ptr(h_maxc), _ptr(status),
                          _ptr(h_status), _ptr(hv_slot), nh, _ptr(hv_c), _ptr(tws), tws.numel(),
                          st)
                del tws
                t_sum = None            # (the optimistic passes' sums, as below)
                if self.opt_passes and self.tile_w not in T15_TILE_W:
                    t_sum = self._empty(NV * T8, torch.int32)
                    _lib.call("dps_ct_tiles_sums", _ptr(h_off), _ptr(h_ent), NV * T8, HW,
                              _ptr(t_sum), st)
                half = (h_off, h_ent, h_maxc, h_status, t_sum)
            else:
                tile_off = self._empty(NV * T + 1, torch.int32)
                tile_maxc = self._empty(NV * T + 1, torch.int32)
                tile_gmin = self._empty(T, torch.int64)
                tile_ent = self._empty(ent_cap, torch.int32)
                status = self._empty(1, torch.int32)
                # (many mids: laid out from one radix sort of (bucket, entry) pairs,
                # dps_ct_tiles_build2; bnd.expand bounds nnz over the author rows)
                tws = self._ws(_lib.size("dps_ct_tiles_workspace_size2", NV, NA, self.tile_w,
                                         bnd.expand))
                _lib.call("dps_ct_tiles_build2", _ptr(c_ptr), _ptr(c_col), _ptr(c_val), _ptr(den),
                          _ptr(t_rank), NA, NV, self.tile_w, bnd.expand, _ptr(tile_off),
                          _ptr(tile_ent), _ptr(tile_maxc), _ptr(tile_gmin), _ptr(status), _ptr(tws),
                          tws.numel(), st)
                del tws
            mark("tiles")
            if not dual and self.tile_w in FOUR_BIT_TILE_W and self.half_tiles:
                # companion u8 tiles at half the width: a tile whose 4-bit bound
                # exceeds 15 runs as its two halves from these (dps_cct_ext)
                HW = self.tile_w // 2
                T8 = max(1, math.ceil(NA / HW)) if NA else 1
                h_cap = _lib.size("dps_ct_tiles_ent_capacity", bnd.expand, bnd.sum_c, NV, NA, HW)
                if split:
                    h_off, h_ent, h_maxc, _, h_status = self._split_tiles(split, sub, HW, g_t,
                                                                          False, h_cap)
                else:
                    h_off = self._empty(NV * T8 + 1, torch.int32)
                    h_maxc = self._empty(NV * T8 + 1, torch.int32)
                    h_ent = self._empty(h_cap, torch.int32)
                    h_status = self._empty(1, torch.int32)
                    hws = self._ws(_lib.size("dps_ct_tiles_workspace_size2", NV, NA, HW,
                                             bnd.expand))
                    _lib.call("dps_ct_tiles_build2", _ptr(c_ptr), _ptr(c_col), _ptr(c_val), None,
                              _ptr(t_rank), NA, NV, HW, bnd.expand, _ptr(h_off), _ptr(h_ent),
                              _ptr(h_maxc), None, _ptr(h_status), _ptr(hws), hws.numel(), st)
                    del hws
                # per-bucket count sums of the companion tiles: the hot kernel's
                # optimistic 4-bit passes check each half's digit sum against
                # them (dps_cct_ext.tile_sum)
                t_sum = None
                if self.opt_passes and self.tile_w not in T15_TILE_W:
                    t_sum = self._empty(NV * T8, torch.int32)
                    _lib.call("dps_ct_tiles_sums", _ptr(h_off), _ptr(h_ent), NV * T8, HW,
                              _ptr(t_sum), st)
                half = (h_off, h_ent, h_maxc, h_status, t_sum)
                mark("half_tiles")
            del sub
            if not dual:
                hv_slot, hv_c, nh = self._heavy_venues(n_v, NA, NV, st)
                if hv_c is not None:
                    _lib.call("dps_heavy_table", _ptr(c_ptr), _ptr(c_col), _ptr(c_val), _ptr(t_rank),
                              NA, _ptr(hv_slot), nh, _ptr(hv_c), st)
                    mark("heavy")
        d.pop("row_work", None)
        d.update(row_terms=terms, ap_ptr=ap_ptr, ap_col=ap_col, px_ptr=px_ptr, px_col=px_col, c_ptr=c_ptr,
                 c_col=c_col, c_val=c_val, c_nnz=c_nnz, s=s, g=g, diag=diag, den=den, g_t=g_t,
                 t_perm=t_perm, t_rank=t_rank, tile_off=tile_off, tile_ent=tile_ent,
                 tile_maxc=tile_maxc, tile_gmin=tile_gmin, stats=stats, status=status,
                 ap_nnz=ap_nnz, px_nnz=px_nnz, sp_status=sp_status, hv_slot=hv_slot, hv_c=hv_c,
                 half_off=half[0] if half else None, half_ent=half[1] if half else None,
                 half_maxc=half[2] if half else None, half_status=half[3] if half else None,
                 tile_sum=half[4] if half else None,
                 topk_ws=self._ws(_lib.size("dps_cct_topk_workspace_size")))
        self._ext = None
        if hv_c is not None or half is not None:
            self._ext = _lib.CctExt(
                _ptr(s) if hv_c is not None else None, _ptr(hv_slot), _ptr(hv_c),
                min(self.n_heavy, 64) if hv_c is not None else 0,
                _ptr(half[0]) if half else None, _ptr(half[1]) if half else None,
                _ptr(half[2]) if half else None, _ptr(half[4]) if half else None)
        self.built = True
        if timed:
            torch.cuda.synchronize(self.device)
            for (a, ea), (b, eb) in zip(marks, marks[1:]):
                info.phase_ms[b] = ea.elapsed_time(eb)
        if check:
            self.check()
        return self

    # ------------------------------------------------- N > 1 tile slices
    def _split_range(self, split):
        """This rank's target labels [l0, l1): tiles_per_rank tiles of tile_w
        (the same count on every rank, the last ranks may hold fewer)."""
        NA = self.typed.n_authors
        T = max(1, math.ceil(NA / self.tile_w)) if NA else 1
        tr = -(-T // split.world)
        l0 = min(NA, split.rank * tr * self.tile_w)
        return l0, min(NA, l0 + tr * self.tile_w), tr

    def _label_rows(self, split, c_ptr, c_col, c_val, t_perm):
        """Sub-C of this rank's labels in label order (dps_label_rows)."""
        l0, l1, _ = self._split_range(split)
        n = l1 - l0
        cap = self.bounds.expand
        sub_ptr = self._empty(n + 1, torch.int64)
        sub_col, sub_val = self._empty(cap, torch.int32), self._empty(cap, torch.int32)
        ws = self._ws(_lib.size("dps_label_rows_workspace_size", n))
        _lib.call("dps_label_rows", _ptr(c_ptr), _ptr(c_col), _ptr(c_val), _ptr(t_perm), l0, l1,
                  _ptr(sub_ptr), _ptr(sub_col), _ptr(sub_val), _ptr(ws), ws.numel(), self.stream)
        return (l0, l1, sub_ptr, sub_col, sub_val)

    def _split_tiles(self, split, sub, W, g_t, gmin, ent_cap):
        """Tiles of width W over this rank's labels (dps_ct_tiles_build2 on the
        sub-C), packed into a slice (dps_tiles_pack), all-gathered, assembled
        into the full layout (dps_tiles_assemble).  The slice's entry capacity
        is the plan in split.caps under this graph's key (_plan_key): the
        largest slice over the ranks, read back and max-reduced once, at the
        first build of the graph (one host sync and one collective); later
        builds of the same graph produce the same slices and reuse it."""
        l0, l1, sub_ptr, sub_col, sub_val = sub
        NA, NV = self.typed.n_authors, self.typed.n_mids
        st = self.stream
        bnd = self.bounds
        _, _, tr_unit = self._split_range(split)
        tr = tr_unit * (self.tile_w // W)
        T = max(1, math.ceil(NA / W)) if NA else 1
        n = l1 - l0
        tl = -(-n // W)
        # (the host bound over the largest range: the local build's capacity)
        loc_cap = _lib.size("dps_ct_tiles_ent_capacity", bnd.expand, bnd.sum_c, NV,
                            tr_unit * self.tile_w, W)
        loc_off = self._empty(NV * tl + 1, torch.int32)
        loc_maxc = self._empty(NV * tl + 1, torch.int32)
        loc_gmin = self._empty(tl, torch.int64) if gmin else None
        loc_ent = self._empty(loc_cap + 4, torch.int32)
        status = torch.zeros(1, dtype=torch.int32, device=self.device)
        if n > 0:
            ws = self._ws(_lib.size("dps_ct_tiles_workspace_size2", NV, n, W, bnd.expand))
            g_ptr = g_t.data_ptr() + 8 * l0 if gmin else None
            _lib.call("dps_ct_tiles_build2", _ptr(sub_ptr), _ptr(sub_col), _ptr(sub_val), g_ptr,
                      None, n, NV, W, bnd.expand, _ptr(loc_off), _ptr(loc_ent), _ptr(loc_maxc),
                      _ptr(loc_gmin), _ptr(status), _ptr(ws), ws.numel(), st)
            del ws
        key = self._plan_key(split, W)
        if key not in split.caps:
            # the gathered slices must all have one size: the largest real slice
            # (not world x the whole graph's bound)
            words = int(loc_off[NV * tl].item()) if tl else 0
            split.caps[key] = (split.allreduce_max(words) + 3) // 4 * 4
        cap = int(split.caps[key])
        words = _lib.size("dps_tiles_slice_words", NV, tr, cap)
        sl = self._empty(words, torch.int32)
        _lib.call("dps_tiles_pack", _ptr(loc_off), _ptr(loc_maxc), _ptr(loc_gmin), _ptr(loc_ent),
                  NV, tl, tr, cap, _ptr(sl), _ptr(status), st)
        gathered = self._empty(split.world * words, torch.int32)
        split.allgather(sl[:words], gathered[: split.world * words])
        off = self._empty(NV * T + 1, torch.int32)
        maxc = self._empty(NV * T + 1, torch.int32)
        gm = self._empty(T, torch.int64) if gmin else None
        ent = self._empty(ent_cap, torch.int32)
        ws = self._ws(_lib.size("dps_tiles_assemble_workspace_size", NV, split.world))
        _lib.call("dps_tiles_assemble", _ptr(gathered), split.world, NV, T, tr, cap, _ptr(off),
                  _ptr(ent), ent.numel(), _ptr(maxc), _ptr(gm), _ptr(status), _ptr(ws), ws.numel(),
                  st)
        return off, ent, maxc, gm, status

    def _plan_key(self, split, W):
        """The split plan's key: the tile width and the graph's shape and host
        bounds (a TileSplit reused for another graph or other bounds
        must not gather with the old graph's capacity)."""
        bnd = self.bounds
        return (int(W), self.typed.n_authors, self.typed.n_mids, int(bnd.expand), int(bnd.sum_c),
                split.world, self.tile_w)

    def check(self):
        """Read the build's statistics back (one synchronisation) and raise if a
        value exceeds the engine's integer widths.  Fills ``info``."""
        if not self.built:
            raise RuntimeError("call build() first")
        d = self._dev
        info = self.info
        status = d["status"] if d.get("half_status") is None else d["status"] | d["half_status"]
        host = torch.cat([d["stats"], d["ap_nnz"], d["px_nnz"], d["c_nnz"][:1],
                          status.to(torch.int64), d["sp_status"].to(torch.int64)]).cpu()
        # nnz over the author rows (C also holds the untyped author_of rows)
        L = _lib.STATS_LEN
        info.max_c = int(host[_lib.STAT_MAX_C])
        info.max_diag = int(host[_lib.STAT_MAX_DIAG])
        info.max_g = int(host[_lib.STAT_MAX_G])
        info.nnz_ap = int(host[L])
        info.nnz_px = int(host[L + 1])
        info.nnz_c = int(host[_lib.STAT_NNZ_C])
        info.expand = int(host[L + 2])         # nnz of C over every AP row
        status_h = int(host[L + 3])
        if int(host[L + 4]) != 0:             # impossible by construction (raw >= distinct)
            raise RuntimeError("a row's SpGEMM expansion exceeds its host bound")
        if status_h == DPS_ERR_OVERFLOW and self.split is not None and self.split.world > 1 \
                and self.info.max_c <= 0xFFFF:
            raise RuntimeError("a tile slice outgrew the gather capacity of the split build's plan")
        if info.expand > self.bounds.sum_c:   # impossible by construction (raw >= distinct)
            raise RuntimeError(f"nnz(C) {info.expand} exceeds its bound {self.bounds.sum_c}")
        if status_h != 0 or info.max_c > 0xFFFF:
            raise OverflowError(f"max C[x,v] = {info.max_c} exceeds the 16-bit tile packing")
        if info.max_diag >= 2 ** 31:
            raise OverflowError(f"max M[x,x] = {info.max_diag} exceeds the int32 accumulators")
        if info.max_g >= 2 ** 52:
            raise OverflowError("g exceeds 2^52: gx+gy would not be exact in fp64")
        if max(info.max_g, info.max_diag).bit_length() > self.bounds.key_bits:
            raise RuntimeError("target-order key bound too small")   # impossible by construction
        self.checked = True
        return info

    # ------------------------------------------------------------- accessors
    def tensor(self, name):
        return self._dev[name]

    def kernel_counts(self):
        """Work counts of the last one-wave hot-kernel launch (its workspace):
        rows dequeued, accumulator passes, 16-byte chunks scattered, candidates
        completed from the heavy-venue table (venue skipping), optimistic 4-bit
        passes that overflowed and ran again as u8 halves."""
        w = self._dev["topk_ws"][:64].view(torch.int64).cpu().tolist()
        return {"dequeued": int(w[0]), "passes": int(w[1]), "chunks": int(w[2]),
                "verified": int(w[3]), "opt_redo": int(w[4])}

    def _ext_arg(self):
        """Host pointer to the dps_cct_ext struct (None = no extension)."""
        if self._ext is None:
            return None
        return C.addressof(self._ext)

    @property
    def n_targets(self):
        return self.typed.n_authors

    def row_work(self):
        """Per-row work estimate of the hot kernel (device int64 [N_A]): the C^T
        entries the row's venues hold, sum_{v in x} n_v, plus half the mean as a
        stand-in for the per-stage fixed cost.  Used to order rows heaviest
        first and to balance row shards across ranks."""
        if "row_work" not in self._dev:
            d = self._dev
            NA = self.typed.n_authors
            with torch.cuda.device(self.device):
                terms = d["row_terms"][:NA]            # from the build's fused walk pass
                d["row_work"] = terms + (terms.sum() // max(NA, 1)) // 2
        return self._dev["row_work"]

    def _heavy_venues(self, n_v, NA, NV, st):
        """Venue skipping: the heavy venues (most author entries) -> hv_slot,
        and the (unfilled) dense table of C over them by target label; (None,
        None, 0) when venue skipping is off."""
        if not (self.venue_skip and self.denominator == "rowsum" and NA and NV):
            return None, None, 0
        nh = min(self.n_heavy, 64)
        hv_slot = self._empty(NV, torch.int32)
        hv_c = self._empty(NA * nh, torch.int16)
        _lib.call("dps_heavy_venues", _ptr(n_v), NV, nh, _ptr(hv_slot), st)
        return hv_slot, hv_c, nh

    # ------------------------------------------------------------------ top-k
    def topk(self, k: int, row_begin: int = 0, row_end: int | None = None, out=None,
             heavy_first: bool = True, split_rows: int | None = None, pieces: int | None = None,
             row_work: torch.Tensor | None = None):
        """★ all-pairs top-k for author rows [row_begin, row_end) (device tensors).

        ``heavy_first`` dequeues the rows in descending ``row_work`` order (LPT),
        so the few very heavy rows do not trail at the end of the launch.  One
        wave owns one row, so the ``split_rows`` heaviest rows of the range are
        further cut into ``pieces`` target-tile ranges each (processed first, in
        the same launch, by separate waves) and their piece lists merged after
        (dps_topk_merge): a single heavy row then no longer bounds the launch --
        which matters most for the small per-rank shards of an N-GPU run.  The
        results are identical either way.  ``row_work`` (int64, one per row of
        the range) replaces the build's ``row_terms`` as the dequeue key."""
        if not self.built:
            raise RuntimeError("call build() first")
        NA = self.typed.n_authors
        row_end = NA if row_end is None else int(row_end)
        R = row_end - row_begin
        d = self._dev
        if R < 0:
            raise ValueError("row_end < row_begin")
        if out is None:
            out = (torch.empty((R, k), dtype=torch.int32, device=self.device),
                   torch.empty((R, k), dtype=torch.int64, device=self.device),
                   torch.empty((R, k), dtype=torch.float64, device=self.device))
        idx, cnt, sc = out
        if R == 0:
            return idx, cnt, sc
        if self.sym and self.tile_w in SYM_TILE_W and row_begin == 0 and row_end == NA:
            return self._topk_sym(k, out)
        T = max(1, math.ceil(NA / self.tile_w))
        M = self.split_rows if split_rows is None else int(split_rows)
        P = min(self.pieces if pieces is None else int(pieces), T, 64)
        if not heavy_first or P < 2 or R <= 4 * M:
            M = 0
        common = (_ptr(d["c_ptr"]), _ptr(d["c_col"]), _ptr(d["c_val"]), _ptr(d["den"]),
                  _ptr(d["g_t"]), _ptr(d["t_perm"]), _ptr(d["t_rank"]), NA, self.typed.n_mids,
                  self.tile_w, _ptr(d["tile_off"]), _ptr(d["tile_ent"]),
                  _ptr(d["tile_maxc"]) if self.tile_skip else None, _ptr(d["tile_gmin"]),
                  self._ext_arg())
        with torch.cuda.device(self.device):
            dq = None
            if heavy_first and R > 1:
                # rows heaviest first by their C^T entry count (log scale, one
                # radix pass), the M heaviest as M*P pieces in front
                dq = torch.empty(R + M * (P - 1), dtype=torch.int32, device=self.device)
                hws = self._ws(_lib.size("dps_heavy_first_workspace_size", R))
                wk = d["row_terms"][row_begin:row_end]
                if row_work is not None:
                    if (row_work.numel() != R or row_work.dtype != wk.dtype
                            or row_work.device != wk.device):
                        raise ValueError("row_work: one int64 per row of the range, on the device")
                    wk = row_work.contiguous()
                _lib.call("dps_heavy_first", _ptr(wk), R,
                          int(row_begin), M, P if M else 1, _ptr(dq), _ptr(hws), hws.numel(),
                          self.stream)
            self._last_dq = dq      # (tools/row_times.py: dequeue slot -> row)
            if M == 0:
                _lib.call("dps_cct_topk", *common, int(row_begin), int(row_end), _ptr(dq),
                          int(k), _ptr(idx), _ptr(cnt), _ptr(sc), _ptr(d["topk_ws"]),
                          d["topk_ws"].numel(), self.stream)
                return idx, cnt, sc
            # piece tile ranges: the same for every split row (cached)
            key = ("pieces", M, P, T)
            if key not in self._piece_cache:
                part = torch.arange(P + 1, device=self.device, dtype=torch.int64) * T // P
                self._piece_cache = {key: (part[:-1].to(torch.int32).repeat(M),
                                           part[1:].to(torch.int32).repeat(M))}
            t0, t1 = self._piece_cache[key]
            n_p = M * P
            pbuf = (torch.empty((n_p, k), dtype=torch.int32, device=self.device),
                    torch.empty((n_p, k), dtype=torch.int64, device=self.device),
                    torch.empty((n_p, k), dtype=torch.float64, device=self.device))
            _lib.call("dps_cct_topk_split", *common, int(row_begin), int(row_end), _ptr(dq),
                      int(dq.numel()), _ptr(t0), _ptr(t1), n_p, _ptr(pbuf[0]), _ptr(pbuf[1]),
                      _ptr(pbuf[2]), int(k), _ptr(idx), _ptr(cnt), _ptr(sc), _ptr(d["topk_ws"]),
                      d["topk_ws"].numel(), self.stream)
            _lib.call("dps_topk_merge", _ptr(pbuf[0]), _ptr(pbuf[1]), _ptr(pbuf[2]), _ptr(dq), M,
                      P, int(k), NA, int(row_begin), _ptr(idx), _ptr(cnt), _ptr(sc), self.stream)
        return idx, cnt, sc

    def _topk_sym(self, k, out, cap=None):
        """dps_cct_sym over every row: the band pass in heavy-first order, then
        the library's own plan, rest pass and merge.  The records emitted are
        checked against the capacity here (one synchronisation), or by
        :meth:`check_sym` when ``defer_checks`` is set; an overflow reruns with
        room for all of them."""
        d = self._dev
        NA = self.typed.n_authors
        idx, cnt, sc = out
        cap = int(cap or max(1, int(self.sym_rec_per_row * NA)))
        with torch.cuda.device(self.device):
            dq = torch.empty(NA, dtype=torch.int32, device=self.device)
            hws = self._ws(_lib.size("dps_heavy_first_workspace_size", NA))
            _lib.call("dps_heavy_first", _ptr(d["row_terms"][:NA]), NA, 0, 0, 1, _ptr(dq), _ptr(hws),
                      hws.numel(), self.stream)
            sws = self._ws(_lib.size("dps_cct_sym_workspace_size", NA, k, cap))
            stat = torch.zeros(1, dtype=torch.int64, device=self.device)
            if self._ext is not None and self._ext.half_ent:
                self._ext_sym = _lib.CctExt(None, None, None, 0, self._ext.half_off,
                                            self._ext.half_ent, self._ext.half_maxc)
                ext = C.addressof(self._ext_sym)
            else:
                ext = None
            _lib.call("dps_cct_sym", _ptr(d["c_ptr"]), _ptr(d["c_col"]), _ptr(d["c_val"]),
                      _ptr(d["den"]), _ptr(d["g_t"]), _ptr(d["t_perm"]), _ptr(d["t_rank"]), NA,
                      self.typed.n_mids, self.tile_w, _ptr(d["tile_off"]), _ptr(d["tile_ent"]),
                      _ptr(d["tile_maxc"]) if self.tile_skip else None, _ptr(d["tile_gmin"]), ext,
                      _ptr(dq), int(self.sym_band), cap, int(k), _ptr(idx), _ptr(cnt), _ptr(sc),
                      _ptr(stat), _ptr(sws), sws.numel(), _ptr(d["topk_ws"]), d["topk_ws"].numel(),
                      self.stream)
            self._sym_stat = (stat, cap, k)
            if not self.defer_checks:
                n_rec = int(stat.item())
                if n_rec > cap:
                    return self._topk_sym(k, out, cap=n_rec + n_rec // 4 + 1024)
        return idx, cnt, sc

    def check_sym(self):
        """Records of the last symmetric launch within capacity (else raise)."""
        if self._sym_stat is None:
            return 0
        stat, cap, _ = self._sym_stat
        n_rec = int(stat.item())
        if n_rec > cap:
            raise RuntimeError(f"symmetric top-k: {n_rec} records exceed the capacity {cap}; "
                               "raise sym_rec_per_row")
        return n_rec

    def topk_rows(self, k: int, rows, out=None):
        """★ top-k of an arbitrary list of author rows (device or host int array),
        one launch, rows dequeued heaviest first; output row i is rows[i]."""
        if not self.built:
            raise RuntimeError("call build() first")
        d = self._dev
        NA = self.typed.n_authors
        rows = torch.as_tensor(rows, device=self.device).to(torch.int64).reshape(-1)
        R = rows.numel()
        if out is None:
            out = (torch.empty((R, k), dtype=torch.int32, device=self.device),
                   torch.empty((R, k), dtype=torch.int64, device=self.device),
                   torch.empty((R, k), dtype=torch.float64, device=self.device))
        if R == 0:
            return out
        with torch.cuda.device(self.device):
            perm = torch.argsort(self.row_work()[rows], descending=True, stable=True)
            order = rows[perm].to(torch.int32)
            tmp = tuple(torch.empty_like(o) for o in out)
            _lib.call("dps_cct_topk_rows", _ptr(d["c_ptr"]), _ptr(d["c_col"]), _ptr(d["c_val"]),
                      _ptr(d["den"]), _ptr(d["g_t"]), _ptr(d["t_perm"]), _ptr(d["t_rank"]), NA,
                      self.typed.n_mids, self.tile_w, _ptr(d["tile_off"]), _ptr(d["tile_ent"]),
                      _ptr(d["tile_maxc"]) if self.tile_skip else None, _ptr(d["tile_gmin"]),
                      self._ext_arg(), _ptr(order), R, int(k), _ptr(tmp[0]), _ptr(tmp[1]), _ptr(tmp[2]),
                      _ptr(d["topk_ws"]), d["topk_ws"].numel(), self.stream)
            for o, t in zip(out, tmp):
                o[perm] = t
        return out

    # -------------------------------------------------------- single source
    def source_row(self, node_index: int):
        """Sparse C row (cols, vals device tensors) of ANY node (DPathSim_APVPA.py:77):
        C is built over every row id, so non-author sources of author_of edges
        have their rows too (empty for nodes without such edges)."""
        d = self._dev
        rid = int(self.typed.node_rowid[node_index])
        b, e = (int(v) for v in d["c_ptr"][rid:rid + 2].cpu())
        return d["c_col"][b:e], d["c_val"][b:e]

    def global_walk(self, node_index: int) -> int:
        """metapath_global_walk (DPathSim_APVPA.py:70-88) for any node."""
        col, val = self.source_row(node_index)
        with torch.cuda.device(self.device):
            ptr = torch.tensor([0, col.numel()], dtype=torch.int64, device=self.device)
            g = self._empty(1, torch.int64)
            _lib.call("dps_global_walks", _ptr(ptr), _ptr(col), _ptr(val), 1, _ptr(self._dev["s"]),
                      _ptr(g), None, None, self.stream)
            return int(g.item())

    def walk_row(self, node_index: int):
        """Dense pairwise walks of one source against every author (int64 device)."""
        col, val = self.source_row(node_index)
        d = self._dev
        NA = self.typed.n_authors
        out = self._empty(NA, torch.int64)
        with torch.cuda.device(self.device):
            _lib.call("dps_walk_row", _ptr(col), _ptr(val), col.numel(), _ptr(d["t_perm"]), NA,
                      self.typed.n_mids,
                      self.tile_w, _ptr(d["tile_off"]), _ptr(d["tile_ent"]), _ptr(out),
                      self.stream)
        return out[:NA]

    def pairwise_walk(self, a_index: int, b_index: int) -> int:
        """metapath_pairwise_walk (DPathSim_APVPA.py:90-109) for any two nodes."""
        ac, av = self.source_row(a_index)
        bc, bv = self.source_row(b_index)
        with torch.cuda.device(self.device):
            out = self._empty(1, torch.int64)
            _lib.call("dps_pair_count", _ptr(ac), _ptr(av), ac.numel(), _ptr(bc), _ptr(bv),
                      bc.numel(), _ptr(out), self.stream)
            return int(out.item())


def host_bounds(typed: TypedTables) -> Bounds:
    """Capacity bounds from the raw typed edges (see :class:`Bounds`)."""
    from . import _lib as L
    g = typed.graph
    NA, NP, NV = typed.n_authors, typed.n_papers, typed.n_mids
    if g.n_edges == 0 or NP == 0:
        return Bounds()   # (max_mids_per_paper 0: the single-mid SpGEMM)
    src, dst, rel = g.edge_src, g.edge_dst, typed.edge_rel
    nt = typed.node_type
    ap = (rel == L.R_AP) & (nt[dst] == L.T_PAPER)
    px = (rel == L.R_PX) & (nt[src] == L.T_PAPER) & (nt[dst] == L.T_MID)
    col = typed.node_colid
    ap_p = col[dst[ap]].astype(np.int64)
    ap_row = typed.node_rowid[src[ap]].astype(np.int64)
    px_p, px_v = col[src[px]].astype(np.int64), col[dst[px]].astype(np.int64)
    pxdeg = np.bincount(px_p, minlength=NP)
    per_edge = pxdeg[ap_p]                                   # raw |PX[p]| per raw AP edge
    is_author = ap_row < NA
    expand = int(per_edge[is_author].sum())
    sum_c = int(per_edge.sum())
    indeg = np.bincount(ap_p, minlength=NP)
    s_max = int(np.bincount(px_v, weights=indeg[px_p], minlength=max(NV, 1)).max()) if len(px_v) else 0
    row_c = np.bincount(ap_row[is_author], weights=per_edge[is_author], minlength=max(NA, 1))
    c_row_max = int(row_c.max()) if NA else 0
    # g[x] <= (sum_v C[x,v]) * max_v s_v;  M[x,x] <= (sum_v C[x,v])^2 <= that too
    gb = max(c_row_max * max(s_max, c_row_max), 1)
    row_all = np.bincount(ap_row, weights=per_edge, minlength=1)
    return Bounds(expand=max(expand, 1), sum_c=max(sum_c, 1), key_bits=min(64, gb.bit_length()),
                  max_row_expand=max(int(row_all.max()), 1),
                  max_mids_per_paper=int(pxdeg.max()) if NP else 0)


def auto_tile_w(typed: TypedTables, bounds: Bounds) -> int:
    """Tile width by shape: 16384 (4-bit counters) when the mean over authors of
    sum_v C[x,v] -- bounded above by the raw expansion count, Bounds.expand --
    is at most AUTO_TILE_W_MAX_ROW_SUM, else 8192 (u8)."""
    na = max(typed.n_authors, 1)
    return 16384 if bounds.expand / na <= AUTO_TILE_W_MAX_ROW_SUM else 8192


def build_engine(typed: TypedTables, device=None, tile_w=DEFAULT_TILE_W, timed=False,
                 denominator="rowsum", spgemm="sort", venue_skip=None):
    t0 = time.perf_counter()
    eng = PathSimEngine(typed, device=device, tile_w=tile_w, denominator=denominator)
    eng.spgemm = spgemm
    if venue_skip is not None:
        eng.venue_skip = bool(venue_skip) and denominator == "rowsum"
    eng.upload()
    eng.build(timed=timed)
    eng.info.phase_ms["host_total"] = (time.perf_counter() - t0) * 1e3
    return eng
