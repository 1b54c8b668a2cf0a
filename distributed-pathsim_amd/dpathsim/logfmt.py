"""All-pairs results in the reference's run-log format (DPathSim_APVPA.py:32-67).

The reference logs one source author's run as ``Source author global walk``
followed by a five-line block per target (``Pairwise authors walk``, ``Target
author global walk``, ``Sim score``, ``***Stage done in``, ``---``).  The
all-pairs engine emits the same blocks for every source row, ranked targets
only, through the native writer ``dps_write_topk_log`` (C++, threaded, Python
``repr`` float formatting) -- formatting 10^7..10^8 target blocks in Python
would take far longer than computing them.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _lib


def format_float(v: float) -> str:
    """Python ``repr(float)`` computed by the native formatter (parity helper)."""
    buf = C.create_string_buffer(64)
    _lib.call("dps_format_float", float(v), buf, 64)
    return buf.value.decode()


class AuthorStrings:
    """UTF-8 node ids and labels of every author ordinal, packed for the writer."""

    def __init__(self, typed):
        g = typed.graph
        nodes = typed.author_nodes.tolist()
        ids = [g.node_id(n).encode("utf-8") for n in nodes]
        labels = [str(g.label(n)).encode("utf-8") for n in nodes]
        self.id_blob, self.id_off = self._pack(ids)
        self.label_blob, self.label_off = self._pack(labels)

    @staticmethod
    def _pack(items):
        off = np.zeros(len(items) + 1, dtype=np.int64)
        if items:
            off[1:] = np.cumsum([len(b) for b in items])
        return b"".join(items), off


def write_topk_log(path, typed, idx, cnt, score, g, row_begin=0, append=True,
                   stage_seconds=0.0, overall_seconds=None, n_threads=0, strings=None):
    """Write source rows [row_begin, row_begin + len(idx)) in the reference log format.

    idx/cnt/score: host arrays [rows, k] (dps_cct_topk output); g: the global
    walks of every author ordinal.  ``stage_seconds`` is written on every
    ``***Stage done in`` line (the per-pair share of the device time);
    ``overall_seconds`` (optional) closes the file like the reference's
    ``***Overall done in`` line.
    """
    idx = np.ascontiguousarray(idx, dtype=np.int32)
    cnt = np.ascontiguousarray(cnt, dtype=np.int64)
    score = np.ascontiguousarray(score, dtype=np.float64)
    g = np.ascontiguousarray(g, dtype=np.int64)
    if idx.ndim != 2 or cnt.shape != idx.shape or score.shape != idx.shape:
        raise ValueError("idx, cnt and score must be [rows, k] arrays of one shape")
    rows, k = idx.shape
    if row_begin < 0 or row_begin + rows > typed.n_authors or len(g) < typed.n_authors:
        raise ValueError("row range or g outside the author ordinals")
    if rows and (idx.max(initial=-1) >= typed.n_authors):
        raise ValueError("target index outside the author ordinals")
    s = strings or AuthorStrings(typed)
    _lib.call("dps_write_topk_log", os.fsencode(path), int(bool(append)), int(row_begin),
              int(rows), int(k), idx.ctypes.data, cnt.ctypes.data, score.ctypes.data,
              g.ctypes.data, s.id_blob, s.id_off.ctypes.data, s.label_blob,
              s.label_off.ctypes.data, float(stage_seconds),
              -1.0 if overall_seconds is None else float(overall_seconds), int(n_threads))
    return s
