"""ORACLE -- TEST INFRASTRUCTURE ONLY.

Literal relational-join restatement of the reference's graphframes motif query
(``DPathSim_APVPA.py:70-109``), used to cross-check ``pathsim_oracle.py`` on
small graphs (including hypothesis-generated multigraphs).

graphframes 0.5.0 (``DPathSim_APVPA.py:147``; not vendored, not available
offline) compiles ``find("(a1)-[e1]->(p1); (p1)-[e2]->(v); (p2)-[e3]->(v);
(a2)-[e4]->(p2)")`` into joins of the edge DataFrame with itself and with the
vertex DataFrame on the named endpoints.  Its published semantics: a motif
row binds every named vertex to a full vertex row and every named edge to a
full edge row; vertex and edge distinctness are NOT enforced.  The reference
then applies the ``.filter`` calls (``:77-84`` / ``:97-105``) and counts
``select('*').distinct()`` (``:86`` / ``:107``) -- i.e. the number of distinct
full rows.  Vertices are rows ``(id, label, node_type)`` and edges rows
``(src, dst, relationship)`` (``:160-163``); edge ids are never passed to
Spark (``:123-124``), so parallel identical edges yield identical rows.
"""
from __future__ import annotations


def motif_count(vertices, edges, author_1, author_2=None):
    vrow = {}
    for v in vertices:                      # vertex DataFrame rows (:161)
        vrow.setdefault(v[0], tuple(v))
    erows = [tuple(e) for e in edges]       # edge DataFrame rows (:163)

    def vtype(n):
        return vrow[n][2] if n in vrow else None

    # e1: (author_1)-[e1]->(paper_1), author_1.id = x, e1 author_of, paper_1 paper
    e1s = [e for e in erows if e[0] == author_1 and e[2] == "author_of"
           and e[0] in vrow and vtype(e[1]) == "paper"]
    # e2 / e3: (paper)-[e]->(venue), submit_at, paper typed, venue typed
    by_venue = {}
    for e in erows:
        if e[2] == "submit_at" and vtype(e[0]) == "paper" and vtype(e[1]) == "venue":
            by_venue.setdefault(e[1], []).append(e)
    by_paper_src = {}
    for e in erows:
        if e[2] == "submit_at" and vtype(e[0]) == "paper" and vtype(e[1]) == "venue":
            by_paper_src.setdefault(e[0], []).append(e)
    # e4: (author_2)-[e4]->(paper_2), author_of (author_2 must be a vertex row)
    e4_by_paper = {}
    for e in erows:
        if e[2] == "author_of" and e[0] in vrow and vtype(e[1]) == "paper":
            if author_2 is None or e[0] == author_2:
                e4_by_paper.setdefault(e[1], []).append(e)

    rows = set()
    for e1 in e1s:
        p1 = e1[1]
        for e2 in by_paper_src.get(p1, []):
            v = e2[1]
            for e3 in by_venue.get(v, []):
                p2 = e3[0]
                for e4 in e4_by_paper.get(p2, []):
                    a2 = e4[0]
                    rows.add((vrow[author_1], e1, vrow[p1], e2, vrow[v], e3,
                              vrow[p2], e4, vrow[a2]))
    return len(rows)
