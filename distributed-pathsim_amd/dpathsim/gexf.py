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


def read_gexf(path, with_stats=False):
    """Parse ``path`` into a :class:`Graph` (strings interned, arrays int32)."""
    node_index = {}
    node_ids, labels, types = [], [], []
    node_attr, edge_attr = {}, {}
    attr_class = None
    directed = True
    e_src, e_dst, e_rel, e_key = [], [], [], []
    e_label_missing = []
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

    n = len(node_ids)
    for i in range(n):
        if types[i] is KeyError:
            raise KeyError("node_type")
    src = np.asarray(e_src, dtype=np.int64)
    dst = np.asarray(e_dst, dtype=np.int64)
    m = len(src)
    if not directed and m:
        a, b = np.minimum(src, dst), np.maximum(src, dst)
        src, dst = a, b
    # multigraph key collapse: (src, dst, id) repeated -> the last data wins, first position kept
    keep = np.ones(m, dtype=bool)
    rel = list(e_rel)
    if m:
        pair = src * n + dst
        order = np.argsort(pair, kind="stable")
        ps = pair[order]
        dup_pairs = np.flatnonzero(ps[1:] == ps[:-1])
        if len(dup_pairs):
            # only pairs that really repeat need the per-key Python check
            seen = {}
            cand = np.unique(np.concatenate([order[dup_pairs], order[dup_pairs + 1]]))
            for j in sorted(cand.tolist()):
                kid = e_key[j]
                if kid is None:
                    continue
                key = (int(src[j]), int(dst[j]), kid)
                if key in seen:
                    # networkx MultiGraph.add_edge does datadict.update(attr): a
                    # repeat without a label keeps the earlier one
                    if rel[j] is not KeyError:
                        rel[seen[key]] = rel[j]
                    keep[j] = False
                else:
                    seen[key] = j
        # adjacency order: by source node order, then first insertion of the pair
        first_seen = np.empty(m, dtype=np.int64)
        _, inv = np.unique(pair, return_inverse=True)
        first_pos = np.full(inv.max() + 1 if m else 0, m, dtype=np.int64)
        np.minimum.at(first_pos, inv, np.arange(m))
        first_seen = first_pos[inv]
        sel = np.flatnonzero(keep)
        ordr = np.lexsort((sel, first_seen[sel], src[sel]))
        sel = sel[ordr]
    else:
        sel = np.zeros(0, dtype=np.int64)
    rel_sel = [rel[j] for j in sel.tolist()]
    for r in rel_sel:
        if r is KeyError:
            raise KeyError("label")
    tnames, tmap = [], {}
    tidx = np.empty(n, dtype=np.int32)
    for i, t in enumerate(types):
        if t not in tmap:
            tmap[t] = len(tnames)
            tnames.append(t)
        tidx[i] = tmap[t]
    rnames, rmap = [], {}
    ridx = np.empty(len(rel_sel), dtype=np.int32)
    for j, r in enumerate(rel_sel):
        if r not in rmap:
            rmap[r] = len(rnames)
            rnames.append(r)
        ridx[j] = rmap[r]
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
