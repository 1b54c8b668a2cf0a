"""ctypes binding of libdpathsim.so (the C ABI declared in include/dpathsim.h).

The product path has no CPU fallback: if the shared library is missing or
fails to load, every entry point raises ``DPSLibraryError``.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DPATHSIM_LIB", os.path.join(_HERE, "libdpathsim.so"))

ABI_VERSION = 4  # DPS_ABI_VERSION in include/dpathsim.h

DPS_OK = 0
DPS_ERR_INVALID = -1
DPS_ERR_HIP = -2
DPS_ERR_WORKSPACE = -3
DPS_ERR_OVERFLOW = -4
DPS_ERR_UNSUPPORTED = -5

T_OTHER, T_AUTHOR, T_PAPER, T_MID = 0, 1, 2, 3
R_OTHER, R_AP, R_PX = 0, 1, 2

STAT_MAX_C, STAT_MAX_DIAG, STAT_MAX_G, STAT_NNZ_C = 0, 1, 2, 3
STATS_LEN = 8

TUNE_WAVES_PER_ROW, TUNE_TILE_BUILD, TUNE_BANK_ORDER, TUNE_LEAN_WPC = 1, 2, 3, 4


class CctExt(C.Structure):
    """struct dps_cct_ext (include/dpathsim.h): venue skipping (s, hv_slot,
    hv_c, n_hv) and the companion u8 tiles of tile_w 16384 (half_*)."""
    _fields_ = [("s", C.c_void_p), ("hv_slot", C.c_void_p), ("hv_c", C.c_void_p),
                ("n_hv", C.c_int32), ("half_off", C.c_void_p), ("half_ent", C.c_void_p),
                ("half_maxc", C.c_void_p), ("tile_sum", C.c_void_p)]

_i32 = C.c_int32
_i64 = C.c_int64
_sz = C.c_size_t
_p = C.c_void_p

# name -> (restype, argtypes); pointer args are passed as integers (device addresses)
SIGNATURES = {
    "dps_abi_version": (C.c_int, []),
    "dps_last_error": (C.c_char_p, []),
    "dps_device_count": (C.c_int, []),
    "dps_extract_incidence": (C.c_int, [_p, _p, _p, _i64, _p, _p, _p, _i64,
                                        _p, _p, _p, _p, _p, _p, _p]),
    "dps_csr_build_workspace_size": (_sz, [_i64, _i64]),
    "dps_csr_build": (C.c_int, [_p, _p, _i64, _p, _i64, _p, _p, _p, _p, _sz, _p]),
    "dps_spgemm_expand_size": (C.c_int, [_p, _p, _p, _i64, _p, _p, _p]),
    "dps_spgemm_workspace_size": (_sz, [_i64, _i64]),
    "dps_spgemm_count": (C.c_int, [_p, _p, _p, _i64, _p, _p, _i64, _p, _p, _p, _p,
                                   _i64, _p, _sz, _p]),
    "dps_spgemm_hash_workspace_size": (_sz, [_i64, _i64]),
    "dps_spgemm_hash": (C.c_int, [_p, _p, _p, _i64, _p, _p, _i64, _p, _p, _p, _p, _p, _p, _sz,
                                  _p]),
    "dps_spgemm_single_workspace_size": (_sz, [_i64, _i64, _i64]),
    "dps_spgemm_single": (C.c_int, [_p, _p, _i64, _i64, _p, _p, _i64, _i64, _p, _p, _p, _p, _p,
                                    _sz, _p]),
    "dps_spgemm_single_map": (C.c_int, [_p, _p, _i64, _i64, _p, _p, _p, _i64, _i64, _p, _p, _p,
                                        _p, _p, _sz, _p]),
    "dps_paper_mid_map": (C.c_int, [_p, _p, _i64, _p, _i64, _p, _p]),
    "dps_gexf_open": (_p, [C.c_char_p, _p]),
    "dps_gexf_info": (_i64, [_p, C.c_int32]),
    "dps_gexf_export": (C.c_int, [_p] + [_p] * 15),
    "dps_gexf_close": (None, [_p]),
    "dps_mid_walks": (C.c_int, [_p, _p, _i64, _p, _p, _i64, _i64, _p, _p, _p]),
    "dps_global_walks": (C.c_int, [_p, _p, _p, _i64, _p, _p, _p, _p, _p]),
    "dps_row_work": (C.c_int, [_p, _p, _i64, _i64, _p, _p, _p]),
    "dps_col_sums": (C.c_int, [_p, _p, _p, _i64, _i64, _p, _p]),
    "dps_walks_fused": (C.c_int, [_p, _p, _p, _i64, _i64, _i64, _p, _p, _p, _p, _p, _p, _p]),
    "dps_walks_fused_ws": (C.c_int, [_p, _p, _p, _i64, _i64, _i64, _p, _p, _p, _p, _p, _p, _i64, _p,
                                     _sz, _p]),
    "dps_walks_workspace_size": (C.c_size_t, [_i64, _i64]),
    "dps_target_order_workspace_size": (_sz, [_i64]),
    "dps_target_order": (C.c_int, [_p, _i64, _i32, _p, _p, _p, _p, _sz, _p]),
    "dps_ct_tiles_workspace_size": (_sz, [_i64, _i64, _i32]),
    "dps_ct_tiles_ent_capacity": (_i64, [_i64, _i64, _i64, _i64, _i32]),
    "dps_ct_tiles_sums": (C.c_int, [_p, _p, _i64, _i32, _p, _p]),
    "dps_ct_tiles_workspace_size2": (_sz, [_i64, _i64, _i32, _i64]),
    "dps_ct_tiles_build2": (C.c_int, [_p, _p, _p, _p, _p, _i64, _i64, _i32, _i64, _p, _p, _p, _p,
                                      _p, _p, _sz, _p]),
    "dps_ct_tiles_build": (C.c_int, [_p, _p, _p, _p, _p, _i64, _i64, _i32, _p, _p, _p, _p, _p,
                                     _p, _sz, _p]),
    "dps_ct_tiles_workspace_size_dual": (_sz, [_i64, _i64, _i32, _i64]),
    "dps_ct_tiles_build_dual": (C.c_int, [_p, _p, _p, _p, _p, _i64, _i64, _i32, _i64, _p, _p, _i64,
                                          _p, _p, _p, _p, _i64, _p, _p, _p, _p, _i32, _p, _p, _sz,
                                          _p]),
    "dps_cct_topk_workspace_size": (_sz, []),
    "dps_cct_topk": (C.c_int, [_p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i32, _p, _p, _p, _p, _p,
                               _i64, _i64, _p, _i32, _p, _p, _p, _p, _sz, _p]),
    "dps_cct_topk_rows": (C.c_int, [_p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i32, _p, _p, _p, _p,
                                    _p, _p, _i64, _i32, _p, _p, _p, _p, _sz, _p]),
    "dps_cct_topk_split": (C.c_int, [_p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i32, _p, _p, _p,
                                     _p, _p, _i64, _i64, _p, _i64, _p, _p, _i64, _p, _p, _p, _i32,
                                     _p, _p, _p, _p, _sz, _p]),
    "dps_cct_sym_workspace_size": (_sz, [_i64, _i32, _i64]),
    "dps_cct_sym": (C.c_int, [_p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i32, _p, _p, _p, _p, _p,
                              _p, _i32, _i64, _i32, _p, _p, _p, _p, _p, _sz, _p, _sz, _p]),
    "dps_heavy_venues": (C.c_int, [_p, _i64, _i32, _p, _p]),
    "dps_heavy_table": (C.c_int, [_p, _p, _p, _p, _i64, _p, _i32, _p, _p]),
    "dps_set_tuning": (C.c_int, [_i32, _i32]),
    "dps_comm_id_bytes": (C.c_int, []),
    "dps_comm_get_id": (C.c_int, [_p]),
    "dps_comm_init": (C.c_int, [_p, _i32, _i32, _p]),
    "dps_comm_destroy": (C.c_int, [_p]),
    "dps_bcast": (C.c_int, [_p, _p, _sz, _i32, _p]),
    "dps_gather": (C.c_int, [_p, _p, _p, _sz, _i32, _p]),
    "dps_allgather": (C.c_int, [_p, _p, _p, _sz, _p]),
    "dps_get_tuning": (C.c_int, [_i32]),
    "dps_shard_edges_workspace_size": (_sz, [_i64]),
    "dps_shard_edges": (C.c_int, [_p, _i64, _i32, _p, _p, _p, _p, _sz, _p]),
    "dps_pack_counts": (C.c_int, [_p, _p, _i64, _p, _p]),
    "dps_unpack_gathered": (C.c_int, [_p, _i32, _i64, _i32, _p, _i64, _p, _p, _p, _p, _p]),
    "dps_label_rows_workspace_size": (_sz, [_i64]),
    "dps_label_rows": (C.c_int, [_p, _p, _p, _p, _i64, _i64, _p, _p, _p, _p, _sz, _p]),
    "dps_tiles_slice_words": (_i64, [_i64, _i64, _i64]),
    "dps_tiles_pack": (C.c_int, [_p, _p, _p, _p, _i64, _i64, _i64, _i64, _p, _p, _p]),
    "dps_tiles_assemble_workspace_size": (_sz, [_i64, _i32]),
    "dps_tiles_assemble": (C.c_int, [_p, _i32, _i64, _i64, _i64, _i64, _p, _p, _i64, _p, _p, _p,
                                     _p, _sz, _p]),
    "dps_topk_merge": (C.c_int, [_p, _p, _p, _p, _i64, _i32, _i32, _i64, _i64, _p, _p, _p, _p]),
    "dps_heavy_first_workspace_size": (_sz, [_i64]),
    "dps_heavy_first": (C.c_int, [_p, _i64, _i64, _i64, _i32, _p, _p, _sz, _p]),
    "dps_walk_row": (C.c_int, [_p, _p, _i64, _p, _i64, _i64, _i32, _p, _p, _p, _p]),
    "dps_row_scores": (C.c_int, [_p, _p, _i64, _i64, _p, _p, _p]),
    "dps_pair_count": (C.c_int, [_p, _p, _i64, _p, _p, _i64, _p, _p]),
    "dps_format_float": (C.c_int, [C.c_double, C.c_char_p, _sz]),
    "dps_write_topk_log": (C.c_int, [C.c_char_p, C.c_int, _i64, _i64, _i32, _p, _p, _p, _p,
                                     C.c_char_p, _p, C.c_char_p, _p, C.c_double, C.c_double,
                                     C.c_int]),
}


class DPSLibraryError(RuntimeError):
    """libdpathsim.so is missing or does not load -- there is no fallback."""


class DPSError(RuntimeError):
    def __init__(self, fn, code, msg):
        super().__init__(f"{fn} failed with status {code}: {msg}")
        self.code = code


_lock = threading.Lock()
_lib = None


def load():
    """Load (once) and return the ctypes handle; raises if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise DPSLibraryError(
                f"{LIB_PATH} not found: build it with `make -C distributed-pathsim_amd/csrc` "
                "or __graft_entry__.build(); the engine has no CPU fallback")
        # torch first: its bundled libamdhip64.so.7 then serves our NEEDED entry,
        # so both share one HIP runtime (same streams, same allocations).
        try:
            import torch  # noqa: F401
        except Exception:  # pragma: no cover - torch is part of the image
            pass
        try:
            lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        except OSError as e:
            raise DPSLibraryError(f"cannot load {LIB_PATH}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.dps_abi_version() != ABI_VERSION:
            raise DPSLibraryError(
                f"{LIB_PATH} has ABI {lib.dps_abi_version()}, the bindings expect {ABI_VERSION}: "
                "rebuild it")
        _lib = lib
        return lib


def exported_symbols():
    return list(SIGNATURES)


def call(name, *args):
    """Call a status-returning entry point; raise DPSError on failure."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != DPS_OK:
        raise DPSError(name, rc, lib.dps_last_error().decode(errors="replace"))
    return rc


def size(name, *args):
    return int(getattr(load(), name)(*args))
