"""Streaming GEXF loader with the reference loader's semantics.

The reference reads the graph with ``networkx.read_gexf`` (a whole-document
DOM parse, ``DPathSim_APVPA.py:116``) and flattens it into vertex tuples
``(id, label, node_type)`` (``:120-121``) and edge tuples ``(src, dst,
d['label'])`` (``:123-124``).  This loader streams the XML with
``xml.etree.ElementTree.iterparse`` (expat; elements are discarded as they
are consumed) and reproduces what networkx 3.4.2's GEXFReader + the reference
loop produce:

* node order = first appearance of each ``<node id>``; a repeated id updates
  the attributes in place; ``data['label']`` is the XML ``label`` attribute
  (it overrides an attvalue titled "label"); ``node_type`` comes from the
  attvalue whose attribute title is ``node_type``.
* edges: attvalues by title, then the XML ``label`` attribute overrides the
  "label" title (= the relationship).  Multigraph keys are the edge ``id``s:
  a repeated (src, dst, id) updates that edge instead of adding one.
  ``type="mutual"`` adds both directions.  Edge iteration order is networkx's
  adjacency order: by source-node order, then first insertion of (src, dst).
* undirected graphs (defaultedgetype != "directed"): networkx's Graph
  iteration reports each edge from its endpoint that comes first in node
  order, so that endpoint becomes ``src`` here too.
* A node referenced only by edges has no ``node_type``: the reference loop
  raises ``KeyError('node_type')``; so does this loader.  Nested ``<nodes>``
  (GEXF sub-nodes) are rejected with NotImplementedError.
"""
from __future__ import annotations

import xml.etree.ElementTree as ET

import numpy as np

from .graph import Graph

_STRINGY = {"string", "liststring", "anyURI"}


def _local(tag):
    return tag.rsplit("}", 1)[-1]


def _convert(value, atype):
    if atype in _STRINGY or atype is None:
        return value
    if atype in ("integer", "long", "short", "byte"):
        return int(value)
    if atype in ("float", "double"):
        return float(value)
    if atype == "boolean":
        return {"true": True, "false": False, "True": True, "False": False, "1": True,
                "0": False}[value]
    return value


def _intern(values, missing):
    """Objects -> (int32 codes in first-appearance order, distinct values);
    ``missing`` (KeyError / None markers) -> -1."""
    table, names = {}, []
    codes = np.empty(len(values), dtype=np.int64)
    for i, v in enumerate(values):
        if v is missing:
            codes[i] = -1
            continue
        c = table.get(v)
        if c is None:
            c = table[v] = len(names)
            names.append(v)
        codes[i] = c
    return codes, names


def _parse_python(path):
    """The iterparse loop (the reference semantics, any GEXF ElementTree reads)."""
    node_index = {}
    node_ids, labels, types = [], [], []
    node_attr, edge_attr = {}, {}
    attr_class = None
    directed = True
    e_src, e_dst, e_rel, e_key = [], [], [], []
    depth_nodes = 0
    cur = None          # dict for the element being assembled
    cur_kind = None

    def node_slot(nid):
        i = node_index.get(nid)
        if i is None:
            i = len(node_ids)
            node_index[nid] = i
            node_ids.append(nid)
            labels.append(None)
            types.append(KeyError)   # marker: no node_type (edge-only node)
        return i

    for ev, el in ET.iterparse(path, events=("start", "end")):
        tag = _local(el.tag)
        if ev == "start":
            if tag == "graph":
                directed = el.get("defaultedgetype") == "directed"
            elif tag == "attributes":
                attr_class = el.get("class")
            elif tag == "nodes":
                depth_nodes += 1
                if depth_nodes > 1:
                    raise NotImplementedError("GEXF sub-nodes (nested <nodes>) are not supported")
            elif tag == "node":
                cur, cur_kind = {"id": el.get("id"), "label": el.get("label"), "att": {}}, "node"
            elif tag == "edge":
                cur, cur_kind = {"src": el.get("source"), "dst": el.get("target"),
                                 "id": el.get("id"), "label": el.get("label"),
                                 "type": el.get("type"), "att": {}}, "edge"
            continue
        # ---- end events
        if tag == "attribute":
            table = node_attr if attr_class == "node" else edge_attr
            table[el.get("id")] = (el.get("title"), el.get("type"))
        elif tag == "attvalue" and cur is not None:
            table = node_attr if cur_kind == "node" else edge_attr
            key = el.get("for")
            if key not in table:
                raise ValueError(f"No attribute defined for={key}.")
            title, atype = table[key]
            cur["att"][title] = _convert(el.get("value"), atype)
        elif tag == "node" and cur_kind == "node":
            i = node_slot(cur["id"])
            labels[i] = cur["label"]
            if "node_type" in cur["att"]:
                types[i] = cur["att"]["node_type"]
            cur, cur_kind = None, None
            el.clear()
        elif tag == "edge" and cur_kind == "edge":
            etype = cur["type"]
            if directed and etype == "undirected":
                raise ValueError("Undirected edge found in directed graph.")
            if (not directed) and etype == "directed":
                raise ValueError("Directed edge found in undirected graph.")
            rel = cur["att"].get("label", KeyError)
            if cur["label"] is not None:
                rel = cur["label"]
            s, t = node_slot(cur["src"]), node_slot(cur["dst"])
            pairs = [(s, t)] + ([(t, s)] if etype == "mutual" else [])
            for (a, b) in pairs:
                e_src.append(a)
                e_dst.append(b)
                e_rel.append(rel)
                e_key.append(cur["id"])
            cur, cur_kind = None, None
            el.clear()
        elif tag == "nodes":
            depth_nodes -= 1

    tcodes, tvals = _intern(types, KeyError)
    rcodes, rnames = _intern(e_rel, KeyError)
    return dict(directed=directed, node_ids=node_ids, labels=labels, node_index=node_index,
                tcodes=tcodes, tvals=tvals, src=np.asarray(e_src, dtype=np.int64),
                dst=np.asarray(e_dst, dtype=np.int64), rcodes=rcodes, rnames=rnames,
                key=e_key.__getitem__)


def _parse_native(path):
    """libdpathsim's mmap'ed scanner (dps_gexf.cpp); None when the file is
    outside its subset (the Python loop then reports the reference's error)."""
    import ctypes as C
    from . import _lib
    try:
        lib = _lib.load()
    except _lib.DPSLibraryError:
        return None
    st = C.c_int32(1)
    h = lib.dps_gexf_open(str(path).encode(), C.byref(st))
    if not h or st.value != 0:
        return None
    try:
        n, m, nt, nr = (lib.dps_gexf_info(h, w) for w in range(4))
        directed = bool(lib.dps_gexf_info(h, 4))
        nb_id, nb_lab, nb_t, nb_r, nb_k = (lib.dps_gexf_info(h, w) for w in range(5, 10))
        id_off, lab_off = np.empty(n + 1, np.int64), np.empty(n + 1, np.int64)
        t_off, r_off = np.empty(nt + 1, np.int64), np.empty(nr + 1, np.int64)
        id_buf, lab_buf = np.empty(max(nb_id, 1), np.uint8), np.empty(max(nb_lab, 1), np.uint8)
        t_buf, r_buf = np.empty(max(nb_t, 1), np.uint8), np.empty(max(nb_r, 1), np.uint8)
        lab_null = np.empty(max(n, 1), np.uint8)
        tcodes = np.empty(max(n, 1), np.int32)
        src, dst = np.empty(max(m, 1), np.int32), np.empty(max(m, 1), np.int32)
        rcodes, koff = np.empty(max(m, 1), np.int32), np.empty(max(m, 1), np.int64)
        kbuf = np.empty(max(nb_k, 1), np.uint8)
        ptr = lambda a: a.ctypes.data
        lib.dps_gexf_export(h, ptr(id_off), ptr(id_buf), ptr(lab_off), ptr(lab_buf), ptr(lab_null),
                            ptr(tcodes), ptr(t_off), ptr(t_buf), ptr(src), ptr(dst), ptr(rcodes),
                            ptr(koff), ptr(kbuf), ptr(r_off), ptr(r_buf))
    finally:
        lib.dps_gexf_close(h)

    def strings(buf, off, k):
        raw = buf[: off[k]].tobytes()
        if raw.isascii():            # byte offsets are character offsets
            text = raw.decode("ascii")
            o = off.tolist()
            return [text[o[i]:o[i + 1]] for i in range(k)]
        o = off.tolist()
        return [raw[o[i]:o[i + 1]].decode("utf-8") for i in range(k)]

    try:
        node_ids = strings(id_buf, id_off, n)
        labels = strings(lab_buf, lab_off, n)
        tvals, rnames = strings(t_buf, t_off, nt), strings(r_buf, r_off, nr)
    except UnicodeDecodeError:
        return None      # not UTF-8 after all: the Python loop decodes it as networkx does
    for i in np.flatnonzero(lab_null[:n]).tolist():
        labels[i] = None
    return dict(directed=directed, node_ids=node_ids, labels=labels,
                node_index=dict(zip(node_ids, range(n))), tcodes=tcodes[:n].astype(np.int64),
                tvals=tvals, src=src[:m].astype(np.int64),
                dst=dst[:m].astype(np.int64), rcodes=rcodes[:m].astype(np.int64),
                rnames=rnames, key=lambda j: _key_at(kbuf, koff, j))


def _key_at(buf, off, j):
    """Edge j's id (bytes) from the native key buffer, None when it has none."""
    o = int(off[j])
    if o < 0:
        return None
    e = o
    while buf[e] != 0:
        e += 1
    return buf[o:e].tobytes()


def _first_appearance(codes):
    """codes (>= 0) -> (dense ids numbered in order of first appearance, the
    original code of each dense id)."""
    if len(codes) == 0:
        return np.zeros(0, np.int32), np.zeros(0, np.int64)
    u, first, inv = np.unique(codes, return_index=True, return_inverse=True)
    rank = np.empty(len(u), np.int64)
    rank[np.argsort(first, kind="stable")] = np.arange(len(u))
    return rank[inv].astype(np.int32), u[np.argsort(first, kind="stable")]


def read_gexf(path, with_stats=False, native=None):
    """Parse ``path`` into a :class:`Graph` (strings interned, arrays int32).

    The per-element scan runs natively (``dps_gexf_open``, an mmap'ed scanner
    in libdpathsim) when the library is present and the file is inside its
    subset, else in the Python iterparse loop; both feed the same networkx
    key-collapse and ordering below.  ``native``: force one (True / False)."""
    P = None
    if native is not False:
        P = _parse_native(path)
        if P is None and native is True:
            raise RuntimeError("native GEXF scan unavailable or outside its subset")
    if P is None:
        P = _parse_python(path)
    node_ids, labels, node_index = P["node_ids"], P["labels"], P["node_index"]
    n = len(node_ids)
    tcodes = P["tcodes"]
    if n and (tcodes < 0).any():
        raise KeyError("node_type")
    src, dst = P["src"], P["dst"]
    rel = P["rcodes"].copy()
    key_of = P["key"]
    m = len(src)
    if not P["directed"] and m:
        a, b = np.minimum(src, dst), np.maximum(src, dst)
        src, dst = a, b
    # multigraph key collapse: (src, dst, id) repeated -> the last data wins, first position kept
    keep = np.ones(m, dtype=bool)
    if m:
        pair = src * n + dst
        order = np.argsort(pair, kind="stable")
        ps = pair[order]
        dup_pairs = np.flatnonzero(ps[1:] == ps[:-1])
        if len(dup_pairs):
            # only pairs that really repeat need the per-key check
            seen = {}
            cand = np.unique(np.concatenate([order[dup_pairs], order[dup_pairs + 1]]))
            for j in sorted(cand.tolist()):
                kid = key_of(j)
                if kid is None:
                    continue
                key = (int(src[j]), int(dst[j]), kid)
                if key in seen:
                    # networkx MultiGraph.add_edge does datadict.update(attr): a
                    # repeat without a label keeps the earlier one
                    if rel[j] >= 0:
                        rel[seen[key]] = rel[j]
                    keep[j] = False
                else:
                    seen[key] = j
        # adjacency order: by source node order, then first insertion of the pair
        _, inv = np.unique(pair, return_inverse=True)
        first_pos = np.full(inv.max() + 1 if m else 0, m, dtype=np.int64)
        np.minimum.at(first_pos, inv, np.arange(m))
        first_seen = first_pos[inv]
        sel = np.flatnonzero(keep)
        ordr = np.lexsort((sel, first_seen[sel], src[sel]))
        sel = sel[ordr]
    else:
        sel = np.zeros(0, dtype=np.int64)
    rel_sel = rel[sel]
    if len(rel_sel) and (rel_sel < 0).any():
        raise KeyError("label")
    tidx, tcode_of = _first_appearance(tcodes)
    tvals = P["tvals"]
    tnames = [tvals[c] for c in tcode_of.tolist()]
    ridx, rcode_of = _first_appearance(rel_sel)
    rnames = [P["rnames"][c] for c in rcode_of.tolist()]
    g = Graph(tidx, [str(t) if not isinstance(t, str) else t for t in tnames],
              src[sel].astype(np.int32), dst[sel].astype(np.int32), ridx, rnames,
              node_ids=node_ids, labels=labels)
    g._id_index = node_index
    return g


def read_dblp_file(path, verbose=True):
    """``read_dblp_nx_file`` (DPathSim_APVPA.py:114-129): graph + the two prints."""
    g = read_gexf(path)
    if verbose:
        print("Total nodes: {}".format(g.n_nodes))
        print("Total edges: {}".format(g.n_edges))
    return g


def write_gexf(graph: Graph, path, name=""):
    """Write a Graph as GEXF 1.2draft in the layout of dblp/dblp_small.gexf.

    Streams line by line (suitable for multi-GB synthetic graphs); the output
    round-trips through :func:`read_gexf` and ``networkx.read_gexf``.
    """
    from xml.sax.saxutils import quoteattr

    with open(path, "w", encoding="utf-8") as f:
        w = f.write
        w("<?xml version='1.0' encoding='utf-8'?>\n")
        w('<gexf version="1.2" xmlns="http://www.gexf.net/1.2draft" '
          'xmlns:xsi="http://www.w3.org/2001/XMLSchema-instance" '
          'xsi:schemaLocation="http://www.w3.org/2001/XMLSchema-instance">\n')
        w(f'  <graph defaultedgetype="directed" mode="static" name={quoteattr(name)}>\n')
        w('    <attributes class="edge" mode="static">\n'
          '      <attribute id="1" title="label" type="string" />\n    </attributes>\n')
        w('    <attributes class="node" mode="static">\n'
          '      <attribute id="0" title="node_type" type="string" />\n    </attributes>\n')
        w("    <nodes>\n")
        tn = graph.type_names
        for i in range(graph.n_nodes):
            w(f"      <node id={quoteattr(graph.node_id(i))} label={quoteattr(graph.label(i))}>\n"
              f"        <attvalues>\n          <attvalue for=\"0\" "
              f"value={quoteattr(tn[graph.node_type_idx[i]])} />\n"
              "        </attvalues>\n      </node>\n")
        w("    </nodes>\n    <edges>\n")
        rn = graph.rel_names
        for j, (s, t, r) in enumerate(zip(graph.edge_src.tolist(), graph.edge_dst.tolist(),
                                          graph.edge_rel_idx.tolist())):
            w(f'      <edge id="{j}" source={quoteattr(graph.node_id(s))} '
              f'target={quoteattr(graph.node_id(t))} weight="1">\n'
              f'        <attvalues>\n          <attvalue for="1" value={quoteattr(rn[r])} />\n'
              "        </attvalues>\n      </edge>\n")
        w("    </edges>\n  </graph>\n</gexf>\n")
