"""Drop-in for the reference's surface (DPathSim_APVPA.py).

``DPathSim_APVPA`` keeps the reference class's constructor shape, methods and
log format (``DPathSim_APVPA.py:7-109``); ``read_dblp_nx_file`` and
``find_author_node_id_by_name`` mirror the script helpers (``:114-137``).
Where the reference ran two Spark motif queries per target, ``run()`` computes
the source's whole pairwise-walk row, every target's global walk and every
score on the GPU in three launches, then writes the same lines in the same
order.  Errors follow the reference: ZeroDivisionError when gx + gy == 0
(``:51-52``), KeyError when the source is not an author (``:56``).
"""
from __future__ import annotations

import timeit

import torch

from . import _lib
from .engine import PathSimEngine, build_engine
from .gexf import read_gexf
from .graph import APVPA, Graph


def read_dblp_nx_file(dblp_graph_file_path, verbose=True):
    """``read_dblp_nx_file`` (DPathSim_APVPA.py:114-129): (graph, vertices, edges)."""
    g = read_gexf(dblp_graph_file_path)
    vertices = g.vertices()
    edges = g.edges()
    if verbose:
        print("Total nodes: {}".format(len(vertices)))
        print("Total edges: {}".format(len(edges)))
    return g, vertices, edges


def find_author_node_id_by_name(dblp_graph: Graph, author_name):
    """First node whose label equals ``author_name``, else None (:132-137)."""
    for i in range(dblp_graph.n_nodes):
        if dblp_graph.label(i) == author_name:
            return dblp_graph.node_id(i)
    return None


class DPathSim_APVPA:
    """Single-source PathSim with the reference's interface and log format.

    ``dblp_graphframe`` is the engine that replaces the GraphFrame: pass a
    built :class:`PathSimEngine` (or None to build one on the current GPU).
    """

    def __init__(self, dblp_graph: Graph, dblp_graphframe, source_author_node_id,
                 output_file_path):
        self.dblp_graph = dblp_graph
        if dblp_graphframe is None:
            dblp_graphframe = build_engine(dblp_graph.typed(APVPA))
        if not isinstance(dblp_graphframe, PathSimEngine):
            raise TypeError("dblp_graphframe must be a dpathsim PathSimEngine (or None)")
        self.dblp_graphframe = dblp_graphframe
        self.source_author_node_id = source_author_node_id

        self.author_sim_scores = {}
        self.author_id_name_maps = {}
        t = dblp_graphframe.typed
        for n in t.author_nodes.tolist():                       # :18-22, node order
            p = dblp_graph.node_id(n)
            if p != self.source_author_node_id:
                self.author_sim_scores.update({p: 1})
            self.author_id_name_maps.update({p: dblp_graph.label(n)})

        self.output_file = open(output_file_path, "a", encoding="utf-8")   # :25
        self.overall_start_time = timeit.default_timer()

    # ---- node id <-> index ------------------------------------------------
    def _index(self, node_id):
        i = self.dblp_graph.index_of(node_id)
        if i is None:
            raise KeyError(node_id)
        return i

    # ---- reference methods ----------------------------------------------------
    def metapath_global_walk(self, start):
        """Global walk of ``start`` (DPathSim_APVPA.py:70-88)."""
        i = self.dblp_graph.index_of(start)
        return 0 if i is None else self.dblp_graphframe.global_walk(i)

    def metapath_pairwise_walk(self, source, target):
        """Pairwise walk source -> target (DPathSim_APVPA.py:90-109)."""
        a, b = self.dblp_graph.index_of(source), self.dblp_graph.index_of(target)
        if a is None or b is None:
            return 0
        return self.dblp_graphframe.pairwise_walk(a, b)

    def _emit(self, line, to_stdout=True):
        if to_stdout:
            print(line)
        self.output_file.write(line + "\n")

    def run(self):
        """DPathSim_APVPA.py:28-68: same prints and log lines, device-computed values.

        The whole source row (pairwise walks, the targets' global walks and the
        scores) is computed on the device up front; the loop below only formats."""
        eng = self.dblp_graphframe
        src = self.source_author_node_id
        gx = self.metapath_global_walk(src)
        self._emit("Source author global walk: {}".format(gx))

        si = self.dblp_graph.index_of(src)
        na = eng.n_targets
        walks = (torch.zeros(na, dtype=torch.int64, device=eng.device) if si is None
                 else eng.walk_row(si))
        g_dev = eng.tensor("g")[:na]
        sc_dev = torch.empty(max(na, 1), dtype=torch.float64, device=eng.device)
        with torch.cuda.device(eng.device):
            _lib.call("dps_row_scores", walks.data_ptr(), g_dev.data_ptr(), int(gx), na,
                      sc_dev.data_ptr(), None, eng.stream)
        walks_h, g_h, sc_h = walks.cpu().tolist(), g_dev.cpu().tolist(), sc_dev[:na].cpu().tolist()
        ordinal_of = {self.dblp_graph.node_id(n): o
                      for o, n in enumerate(eng.typed.author_nodes.tolist())}
        names = self.author_id_name_maps

        for tgt in self.author_sim_scores.keys():                         # :36 target order
            t_start = timeit.default_timer()
            o = ordinal_of[tgt]
            self._emit("Pairwise authors walk {}: {}".format(tgt, int(walks_h[o])))
            gy = int(g_h[o])
            self._emit("Target author global walk: {}".format(gy))
            if gx + gy == 0:
                raise ZeroDivisionError("division by zero")               # :51-52
            self.author_sim_scores[tgt] = sc_h[o]
            # names[src] raises KeyError for a non-author source, as :56 does
            self._emit("Sim score {} - {}: {}".format(names[src], names[tgt], sc_h[o]))
            self._emit("***Stage done in: {}".format(timeit.default_timer() - t_start), False)
            self._emit("---", False)
            self.output_file.flush()

        self._emit("***Overall done in: {}".format(timeit.default_timer() - self.overall_start_time),
                   False)
        self.output_file.close()
