"""ORACLE -- TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference's APVPA PathSim semantics
(phamtheanhphu/Distributed-PathSim, ``DPathSim_APVPA.py``).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker.  The product path
(``distributed-pathsim_amd/dpathsim``) never imports it.

Parity pinning: the reference (pyspark + graphframes 0.5.0, JVM, fetched over the
network at run time, ``DPathSim_APVPA.py:146-148``) cannot run in this image
(``ModuleNotFoundError: pyspark`` -- an ordinary import error, not a denial).
This restatement is pinned instead by the reference's own recorded outputs:
the 81 (pairwise walk, target global walk, score) triples and the 26 target
global walks of ``output/d_pathsim_output_20180417_020445.log`` that are
reproducible on ``dblp/dblp_small.gexf`` (see ``tests/golden/make_golden.py``),
and by ``motif_bruteforce.py``, a literal relational-join restatement of the
graphframes motif + filters + ``distinct().count()``.

Semantics restated (all cites are into /root/reference):

* Input schema = what ``read_dblp_nx_file`` hands to Spark
  (``DPathSim_APVPA.py:114-129``, ``:160-163``): vertices ``(id, label,
  node_type)`` and edges ``(src, dst, relationship)``.
* Motif ``(a1)-[e1]->(p1); (p1)-[e2]->(v); (p2)-[e3]->(v); (a2)-[e4]->(p2)``
  with filters ``:77-84`` / ``:97-105``: ``e1,e4`` relationship ``author_of``
  with a *paper*-typed destination (the source type is NOT checked); ``e2,e3``
  relationship ``submit_at`` from a paper-typed node to a venue-typed node.
  ``select('*').distinct()`` (``:86,107``) makes every incidence binary.
* ``C[a, v] = |{p : (a,p) in AP, (p,v) in PV}|``;
  pairwise walk ``M[x, y] = C[x,:] . C[y,:]`` (``:90-109``);
  global walk ``g[x] = sum_y M[x, y] = C[x,:] . s`` with ``s = colsum(C)`` over
  EVERY AP source (``:70-88``; author_2 is unconstrained, so it includes x).
* Score ``2*M / (gx + gy)`` (``:51-52``): Python int/int true division, i.e. one
  correctly-rounded IEEE fp64 division (== ``float(2M)/float(gx+gy)`` for
  operands below 2**53).
* Targets: ``node_type == 'author'`` nodes in node order, minus the source
  (``:18-22``, loop ``:36``).
* All-pairs top-k (the build's generalisation): for every author
  source x, targets ordered by (score desc, author ordinal asc), first k.
  A pair with gx + gy == 0 (two authors with no walks) scores 0.0 here; the
  reference's single-source ``run()`` would raise ZeroDivisionError and the
  compat class in the product does the same.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

AUTHOR_OF = "author_of"
SUBMIT_AT = "submit_at"


def load_gexf_networkx(path):
    """Reference loader semantics (``DPathSim_APVPA.py:114-129``) via networkx."""
    import networkx as nx

    g = nx.read_gexf(path)
    vertices = [(p, d["label"], d["node_type"]) for p, d in g.nodes(data=True)]
    edges = [(s, t, d["label"]) for s, t, d in g.edges(data=True)]
    return vertices, edges


class OracleGraph:
    """Typed incidence + commuting counts for one meta-path A-P-X-P-A.

    ``mid_type``/``rel_px`` default to APVPA (venue, submit_at); APTPA uses
    ``mid_type='topic'`` and the build's documented relationship name.
    """

    def __init__(self, vertices, edges, author_type="author", paper_type="paper",
                 mid_type="venue", rel_ap=AUTHOR_OF, rel_px=SUBMIT_AT):
        self.node_ids = [v[0] for v in vertices]
        self.labels = {v[0]: v[1] for v in vertices}
        self.types = {v[0]: v[2] for v in vertices}
        idx = {}
        for i, nid in enumerate(self.node_ids):
            idx.setdefault(nid, i)
        self.authors = [v[0] for v in vertices if v[2] == author_type]
        self.author_ord = {a: i for i, a in enumerate(self.authors)}
        self.papers = [v[0] for v in vertices if v[2] == paper_type]
        self.paper_ord = {p: i for i, p in enumerate(self.papers)}
        self.mids = [v[0] for v in vertices if v[2] == mid_type]
        self.mid_ord = {m: i for i, m in enumerate(self.mids)}
        # distinct typed incidences (motif filters :78-84, distinct :86)
        ap, px = set(), set()
        for s, t, r in edges:
            if r == rel_ap and s in self.types and self.types.get(t) == paper_type:
                ap.add((s, t))
            if r == rel_px and self.types.get(s) == paper_type and self.types.get(t) == mid_type:
                px.add((s, t))
        self.ap = ap
        self.px = px
        # every AP source gets a row: authors first (node order), then others (node order)
        srcs = {s for s, _ in ap}
        others = [n for n in self.node_ids if n in srcs and self.types.get(n) != author_type]
        self.rows = list(self.authors) + others
        self.row_ord = {r: i for i, r in enumerate(self.rows)}
        n_r, n_p, n_m = len(self.rows), len(self.papers), len(self.mids)
        if ap:
            ri = np.array([self.row_ord[s] for s, _ in ap], dtype=np.int64)
            pi = np.array([self.paper_ord[t] for _, t in ap], dtype=np.int64)
        else:
            ri = pi = np.zeros(0, dtype=np.int64)
        w_ap = sp.csr_matrix((np.ones(len(ri), dtype=np.int64), (ri, pi)), shape=(n_r, n_p))
        if px:
            qi = np.array([self.paper_ord[s] for s, _ in px], dtype=np.int64)
            mi = np.array([self.mid_ord[t] for _, t in px], dtype=np.int64)
        else:
            qi = mi = np.zeros(0, dtype=np.int64)
        w_px = sp.csr_matrix((np.ones(len(qi), dtype=np.int64), (qi, mi)), shape=(n_p, n_m))
        c_all = (w_ap @ w_px).tocsr()
        c_all.sort_indices()
        c_all.eliminate_zeros()
        self.c_all = c_all
        self.s = np.asarray(c_all.sum(axis=0)).ravel().astype(np.int64)      # s = colsum(C)
        self.g_all = np.asarray(c_all @ self.s).ravel().astype(np.int64)     # g = C . s
        na = len(self.authors)
        self.C = c_all[:na].tocsr()
        self.g = self.g_all[:na].copy()

    # ---- per-node walks (reference methods :70-109) -------------------------
    def crow(self, node_id):
        r = self.row_ord.get(node_id)
        if r is None:
            return sp.csr_matrix((1, self.c_all.shape[1]), dtype=np.int64)
        return self.c_all[r]

    def global_walk(self, node_id):
        """``metapath_global_walk`` (:70-88)."""
        return int((self.crow(node_id) @ self.s)[0])

    def pairwise_walk(self, source, target):
        """``metapath_pairwise_walk`` (:90-109)."""
        return int(self.crow(source).multiply(self.crow(target)).sum())

    def score(self, source, target):
        """Score exactly as :51-52 (raises ZeroDivisionError like the reference)."""
        pw = self.pairwise_walk(source, target)
        return 2 * pw / (self.global_walk(source) + self.global_walk(target))

    # ---- all-pairs -----------------------------------------------------------
    def walk_rows(self, rows):
        """Dense M[rows, authors] as int64 (rows are author ordinals)."""
        blk = (self.C[rows] @ self.C.T).toarray().astype(np.int64)
        return blk


def scores_fp64(m, gx, gy):
    """Element-wise ``2*M/(gx+gy)`` in fp64 (:51-52); 0/0 -> 0.0 (see header)."""
    num = (2 * np.asarray(m, dtype=np.int64)).astype(np.float64)
    den = (np.asarray(gx, dtype=np.int64) + np.asarray(gy, dtype=np.int64)).astype(np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        out = num / den
    out[den == 0] = 0.0
    return out


def allpairs_topk(graph: OracleGraph, k: int, rows=None, block: int = 512,
                  denominator: str = "rowsum"):
    """Top-k per author source by (score desc, author ordinal asc), self excluded.

    ``denominator='rowsum'`` is the reference's 2M/(g[x]+g[y]) (K2); ``'diag'``
    the textbook 2M/(M[x,x]+M[y,y]) that the CLI offers as an option.

    Returns (idx int32[R,k], cnt int64[R,k], score f64[R,k]); slots beyond the
    number of available targets hold idx -1, cnt 0, score 0.0.
    """
    na = len(graph.authors)
    if rows is None:
        rows = np.arange(na)
    rows = np.asarray(rows, dtype=np.int64)
    R = len(rows)
    idx = np.full((R, k), -1, dtype=np.int32)
    cnt = np.zeros((R, k), dtype=np.int64)
    sc = np.zeros((R, k), dtype=np.float64)
    if denominator == "rowsum":
        g = graph.g
    elif denominator == "diag":
        g = np.asarray(graph.C.multiply(graph.C).sum(axis=1)).ravel().astype(np.int64)
    else:
        raise ValueError(denominator)
    ar = np.arange(na)
    for b0 in range(0, R, block):
        rb = rows[b0:b0 + block]
        m = graph.walk_rows(rb)
        s = scores_fp64(m, g[rb][:, None], g[None, :])
        for i, x in enumerate(rb):
            keep = ar != x
            ys = ar[keep]
            ss = s[i, keep]
            order = np.lexsort((ys, -ss))[:k]
            n = len(order)
            idx[b0 + i, :n] = ys[order]
            cnt[b0 + i, :n] = m[i, keep][order]
            sc[b0 + i, :n] = ss[order]
    return idx, cnt, sc


def single_source_log_lines(graph: OracleGraph, source_id: str):
    """Lines of ``run()`` (:28-68) for one source, timing lines omitted."""
    gx = graph.global_walk(source_id)
    out = [f"Source author global walk: {gx}"]
    src_label = graph.labels[source_id] if graph.types.get(source_id) == "author" else None
    for t in graph.authors:
        if t == source_id:
            continue
        pw = graph.pairwise_walk(source_id, t)
        gy = graph.global_walk(t)
        out.append(f"Pairwise authors walk {t}: {pw}")
        out.append(f"Target author global walk: {gy}")
        score = 2 * pw / (gx + gy)
        if src_label is None:
            raise KeyError(source_id)
        out.append(f"Sim score {src_label} - {graph.labels[t]}: {score}")
    return out


# ---------------------------------------------------------------------------
# ctypes wrapper of the C restatement (oracle/pathsim_oracle.c, liboracle.so)
class COracle:
    """C/OpenMP restatement over typed int arrays (same semantics as above)."""

    def __init__(self, ap_row, ap_col, px_paper, px_mid, n_rows_all, n_authors, n_papers, n_mids):
        import ctypes as C
        import os
        here = os.path.dirname(os.path.abspath(__file__))
        path = os.path.join(here, "liboracle.so")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        lib = C.CDLL(path)
        P, I64 = C.c_void_p, C.c_int64
        lib.orc_create.restype = P
        lib.orc_create.argtypes = [I64, P, P, I64, P, P, I64, I64, I64, I64]
        lib.orc_nnz.restype = I64
        lib.orc_nnz.argtypes = [P]
        lib.orc_export.argtypes = [P, P, P, P, P, P]
        lib.orc_topk.argtypes = [P, I64, I64, C.c_int, P, P, P, C.c_int]
        lib.orc_topk_rows.argtypes = [P, P, I64, I64, C.c_int, P, P, P, C.c_int, C.c_int]
        lib.orc_diag.argtypes = [P, P]
        lib.orc_destroy.argtypes = [P]
        lib.orc_set_flags.argtypes = [C.c_int]
        lib.orc_get_flags.restype = C.c_int
        lib.orc_narrow.restype = C.c_int
        lib.orc_narrow.argtypes = [P]
        self._lib = lib
        a = [np.ascontiguousarray(x, dtype=np.int32) for x in (ap_row, ap_col, px_paper, px_mid)]
        self._keep = a
        self.n_authors, self.n_mids = int(n_authors), int(n_mids)
        self._st = lib.orc_create(len(a[0]), a[0].ctypes.data, a[1].ctypes.data, len(a[2]),
                                  a[2].ctypes.data, a[3].ctypes.data, int(n_rows_all),
                                  int(n_authors), int(n_papers), int(n_mids))

    @classmethod
    def from_typed(cls, typed):
        """From dpathsim.graph.TypedTables-like arrays (node tables + edges)."""
        g = typed.graph
        ap = (typed.edge_rel == 1) & (typed.node_type[g.edge_dst] == 2)
        px = ((typed.edge_rel == 2) & (typed.node_type[g.edge_src] == 2)
              & (typed.node_type[g.edge_dst] == 3))
        return cls(typed.node_rowid[g.edge_src[ap]], typed.node_colid[g.edge_dst[ap]],
                   typed.node_colid[g.edge_src[px]], typed.node_colid[g.edge_dst[px]],
                   getattr(typed, "n_rows", g.n_nodes), typed.n_authors, typed.n_papers,
                   typed.n_mids)

    def export(self):
        nnz = self._lib.orc_nnz(self._st)
        c_ptr = np.zeros(self.n_authors + 1, np.int64)
        c_col = np.zeros(max(nnz, 1), np.int32)
        c_val = np.zeros(max(nnz, 1), np.int32)
        s = np.zeros(max(self.n_mids, 1), np.int64)
        g = np.zeros(max(self.n_authors, 1), np.int64)
        self._lib.orc_export(self._st, c_ptr.ctypes.data, c_col.ctypes.data, c_val.ctypes.data,
                             s.ctypes.data, g.ctypes.data)
        return c_ptr, c_col[:nnz], c_val[:nnz], s[: self.n_mids], g[: self.n_authors]

    def topk(self, k, row_begin=0, row_end=None, threads=0):
        row_end = self.n_authors if row_end is None else row_end
        R = row_end - row_begin
        idx = np.zeros((R, k), np.int32)
        cnt = np.zeros((R, k), np.int64)
        sc = np.zeros((R, k), np.float64)
        self._lib.orc_topk(self._st, row_begin, row_end, k, idx.ctypes.data, cnt.ctypes.data,
                           sc.ctypes.data, int(threads))
        return idx, cnt, sc

    def topk_rows(self, k, rows, threads=0, denominator="rowsum"):
        """Top-k of the author rows listed in ``rows`` (any order, output row i is
        rows[i]); ``denominator='diag'`` scores 2M/(M[x,x]+M[y,y]) instead of the
        reference's row sums."""
        rows = np.ascontiguousarray(rows, dtype=np.int64)
        R = len(rows)
        idx = np.zeros((R, k), np.int32)
        cnt = np.zeros((R, k), np.int64)
        sc = np.zeros((R, k), np.float64)
        if denominator not in ("rowsum", "diag"):
            raise ValueError(denominator)
        if R:
            self._lib.orc_topk_rows(self._st, rows.ctypes.data, R, 0, k, idx.ctypes.data,
                                    cnt.ctypes.data, sc.ctypes.data, int(threads),
                                    int(denominator == "diag"))
        return idx, cnt, sc

    # test switches of the C restatement (pathsim_oracle.c: ORC_FORCE_I64,
    # ORC_NO_SKIP); process-wide, tests restore 0 afterwards
    FORCE_I64, NO_SKIP = 1, 2

    def set_flags(self, flags):
        self._lib.orc_set_flags(int(flags))

    def narrow(self):
        """True when topk() runs on int32 accumulators under the current flags."""
        return bool(self._lib.orc_narrow(self._st))

    def diag(self):
        d = np.zeros(max(self.n_authors, 1), np.int64)
        self._lib.orc_diag(self._st, d.ctypes.data)
        return d[: self.n_authors]

    def __del__(self):
        st = getattr(self, "_st", None)
        if st:
            self._lib.orc_destroy(st)
            self._st = None
