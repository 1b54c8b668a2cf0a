"""Host-side typed graph: the arrays the device pipeline consumes.

Mirrors the schema the reference hands to Spark (``DPathSim_APVPA.py:160-163``):
vertices ``(id, label, node_type)`` in node order and edges ``(src, dst,
relationship)``.  Strings are interned once into small integer tables so the
device only ever sees int32/uint8 arrays.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _lib


@dataclass(frozen=True)
class MetaPath:
    """A symmetric A-P-X-P-A meta-path (the motif of DPathSim_APVPA.py:72-84).

    APVPA is the reference's (venue, 'submit_at').  The reference defines no
    relationship for topics (dblp_small has topic nodes but no topic edges,
    SURVEY.md §8d config 4), so APTPA uses the build's own name 'has_topic'.
    """
    name: str = "APVPA"
    author_type: str = "author"
    paper_type: str = "paper"
    mid_type: str = "venue"
    rel_ap: str = "author_of"
    rel_px: str = "submit_at"


APVPA = MetaPath()
APTPA = MetaPath(name="APTPA", mid_type="topic", rel_px="has_topic")
METAPATHS = {"APVPA": APVPA, "APTPA": APTPA}


class Graph:
    """Vertices + edges with interned type/relationship strings.

    node_type_idx[n] indexes ``type_names``; edge_rel_idx[e] indexes
    ``rel_names``.  ``node_ids``/``labels`` are lists of str, or callables
    ``f(i) -> str`` for generated graphs (materialised only when asked).
    """

    def __init__(self, node_type_idx, type_names, edge_src, edge_dst, edge_rel_idx, rel_names,
                 node_ids=None, labels=None):
        self.node_type_idx = np.ascontiguousarray(node_type_idx, dtype=np.int32)
        self.type_names = list(type_names)
        self.edge_src = np.ascontiguousarray(edge_src, dtype=np.int32)
        self.edge_dst = np.ascontiguousarray(edge_dst, dtype=np.int32)
        self.edge_rel_idx = np.ascontiguousarray(edge_rel_idx, dtype=np.int32)
        self.rel_names = list(rel_names)
        self._node_ids = node_ids
        self._labels = labels
        self._id_index = None
        n = len(self.node_type_idx)
        if len(self.edge_src) != len(self.edge_dst) or len(self.edge_src) != len(self.edge_rel_idx):
            raise ValueError("edge arrays differ in length")
        if len(self.edge_src) and (self.edge_src.min() < 0 or self.edge_src.max() >= n
                                   or self.edge_dst.min() < 0 or self.edge_dst.max() >= n):
            raise ValueError("edge endpoint outside the vertex table")

    # ---- construction ----------------------------------------------------
    @classmethod
    def from_tuples(cls, vertices, edges):
        """From the reference loader's lists (DPathSim_APVPA.py:120-124)."""
        ids = [v[0] for v in vertices]
        index = {}
        for i, nid in enumerate(ids):
            index.setdefault(nid, i)
        tnames, tmap = [], {}
        tidx = np.empty(len(vertices), dtype=np.int32)
        for i, v in enumerate(vertices):
            t = v[2]
            if t not in tmap:
                tmap[t] = len(tnames)
                tnames.append(t)
            tidx[i] = tmap[t]
        rnames, rmap = [], {}
        es = np.empty(len(edges), dtype=np.int32)
        ed = np.empty(len(edges), dtype=np.int32)
        er = np.empty(len(edges), dtype=np.int32)
        for j, (s, t, r) in enumerate(edges):
            if s not in index or t not in index:
                # the reference loader raises KeyError on d['node_type'] for such nodes
                raise KeyError(s if s not in index else t)
            es[j] = index[s]
            ed[j] = index[t]
            if r not in rmap:
                rmap[r] = len(rnames)
                rnames.append(r)
            er[j] = rmap[r]
        g = cls(tidx, tnames, es, ed, er, rnames, node_ids=ids, labels=[v[1] for v in vertices])
        g._id_index = index
        return g

    # ---- accessors ---------------------------------------------------------
    @property
    def n_nodes(self):
        return len(self.node_type_idx)

    @property
    def n_edges(self):
        return len(self.edge_src)

    def node_id(self, i):
        ids = self._node_ids
        return ids(i) if callable(ids) else ids[i]

    def label(self, i):
        lab = self._labels
        return lab(i) if callable(lab) else lab[i]

    def node_type(self, i):
        return self.type_names[self.node_type_idx[i]]

    def index_of(self, node_id):
        if self._id_index is None:
            self._id_index = {}
            for i in range(self.n_nodes):
                self._id_index.setdefault(self.node_id(i), i)
        return self._id_index.get(node_id)

    def vertices(self):
        """(id, label, node_type) tuples in node order (DPathSim_APVPA.py:120-121)."""
        return [(self.node_id(i), self.label(i), self.node_type(i)) for i in range(self.n_nodes)]

    def edges(self):
        """(src, dst, relationship) tuples (DPathSim_APVPA.py:123-124)."""
        return [(self.node_id(s), self.node_id(t), self.rel_names[r])
                for s, t, r in zip(self.edge_src.tolist(), self.edge_dst.tolist(),
                                   self.edge_rel_idx.tolist())]

    # ---- typed tables for one meta-path --------------------------------------
    def typed(self, mp: MetaPath = APVPA):
        return TypedTables(self, mp)


class TypedTables:
    """Device-ready index spaces for one meta-path (see include/dpathsim.h)."""

    def __init__(self, graph: Graph, mp: MetaPath):
        self.graph = graph
        self.metapath = mp
        code_of_type = np.zeros(max(1, len(graph.type_names)), dtype=np.uint8)
        for i, t in enumerate(graph.type_names):
            if t == mp.author_type:
                code_of_type[i] = _lib.T_AUTHOR
            elif t == mp.paper_type:
                code_of_type[i] = _lib.T_PAPER
            elif t == mp.mid_type:
                code_of_type[i] = _lib.T_MID
        ntype = code_of_type[graph.node_type_idx] if graph.n_nodes else np.zeros(0, np.uint8)
        self.node_type = np.ascontiguousarray(ntype, dtype=np.uint8)
        is_author = self.node_type == _lib.T_AUTHOR
        is_paper = self.node_type == _lib.T_PAPER
        is_mid = self.node_type == _lib.T_MID
        self.author_nodes = np.flatnonzero(is_author).astype(np.int64)   # author ordinal -> node
        self.n_authors = int(is_author.sum())
        self.n_papers = int(is_paper.sum())
        self.n_mids = int(is_mid.sum())
        colid = np.full(graph.n_nodes, -1, dtype=np.int64)
        colid[is_paper] = np.arange(self.n_papers)
        colid[is_mid] = np.arange(self.n_mids)
        self.node_colid = colid.astype(np.int32)
        rel_code = np.zeros(max(1, len(graph.rel_names)), dtype=np.uint8)
        for i, r in enumerate(graph.rel_names):
            if r == mp.rel_ap:
                rel_code[i] = _lib.R_AP
            elif r == mp.rel_px:
                rel_code[i] = _lib.R_PX
        self.edge_rel = np.ascontiguousarray(
            rel_code[graph.edge_rel_idx] if graph.n_edges else np.zeros(0, np.uint8),
            dtype=np.uint8)
        # C row space: authors [0, N_A) in node order, then the other sources
        # of AP incidences (author_of edges into a paper; the source type is not
        # checked, DPathSim_APVPA.py:78-84) in node order, then ONE shared empty
        # row for every node that can have no C entries -- so the device build's
        # row-indexed passes run over N_A + K + 1 rows, not over every node.
        is_src = np.zeros(graph.n_nodes, dtype=bool)
        if graph.n_edges:
            ap = (self.edge_rel == _lib.R_AP) & is_paper[graph.edge_dst]
            is_src[graph.edge_src[ap]] = True
        other = is_src & ~is_author
        n_other = int(other.sum())
        rowid = np.full(graph.n_nodes, self.n_authors + n_other, dtype=np.int64)
        rowid[is_author] = np.arange(self.n_authors)
        rowid[other] = self.n_authors + np.arange(n_other)
        self.node_rowid = rowid.astype(np.int32)
        self.n_rows = self.n_authors + n_other + 1
        if graph.n_nodes >= 2 ** 31 - 1:
            raise OverflowError("more than 2^31-1 nodes")

    def author_ordinal(self, node_index):
        """Author ordinal of a node index, or None if not author-typed."""
        if self.node_type[node_index] != _lib.T_AUTHOR:
            return None
        return int(self.node_rowid[node_index])
