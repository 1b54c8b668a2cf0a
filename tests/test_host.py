"""CPU: host logic of the product package (loader, typed tables, generator, C ABI)."""
import ctypes
import ctypes as C
import os
import re

import numpy as np
import pytest

from dpathsim import _lib
from dpathsim.gexf import read_gexf, write_gexf
from dpathsim.graph import APTPA, APVPA, Graph
from dpathsim.synth import synth_dblp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_GEXF = "/root/reference/dblp/dblp_small.gexf"


def test_header_symbols_exported():
    """libdpathsim.so loads and exports every function include/dpathsim.h declares."""
    hdr = open(os.path.join(REPO, "include", "dpathsim.h")).read()
    declared = set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\**\s+\**(dps_[a-z_0-9]+)\(", hdr, re.M))
    assert len(declared) >= 15
    lib = _lib.load()
    for name in declared:
        assert hasattr(lib, name), name
    assert set(_lib.exported_symbols()) == declared
    assert lib.dps_abi_version() == 4


def test_no_cpu_fallback_when_library_missing(monkeypatch):
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", "/nonexistent/libdpathsim.so")
    with pytest.raises(_lib.DPSLibraryError):
        _lib.load()


def test_engine_refuses_without_gpu(dblp_small_tuples):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from dpathsim.engine import PathSimEngine
    t = Graph.from_tuples(*dblp_small_tuples).typed()
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        PathSimEngine(t)


def test_typed_tables_dblp_small(dblp_small_tuples):
    v, e = dblp_small_tuples
    g = Graph.from_tuples(v, e)
    t = g.typed(APVPA)
    assert (t.n_authors, t.n_papers, t.n_mids) == (770, 1001, 85)
    authors = [x[0] for x in v if x[2] == "author"]
    assert [g.node_id(int(i)) for i in t.author_nodes] == authors
    # C row space: authors first (node order), then the other AP sources, then
    # one shared empty row for every other node
    assert np.array_equal(t.node_rowid[t.author_nodes], np.arange(770))
    ap = (t.edge_rel == _lib.R_AP) & (t.node_type[np.asarray(g.edge_dst)] == _lib.T_PAPER)
    srcs = np.unique(np.asarray(g.edge_src)[ap])
    assert len(np.unique(t.node_rowid[srcs])) == len(srcs)
    rest = np.setdiff1d(np.arange(g.n_nodes), np.concatenate([srcs, t.author_nodes]))
    assert (t.node_rowid[rest] == t.n_rows - 1).all()
    assert t.n_rows == 770 + len(np.setdiff1d(srcs, t.author_nodes)) + 1
    assert int((t.edge_rel == _lib.R_AP).sum()) == 1265
    assert int((t.edge_rel == _lib.R_PX).sum()) == 1001
    assert g.vertices() == v and g.edges() == e


def test_aptpa_codes():
    g = synth_dblp(50, 100, 20, seed=1, metapath=APTPA)
    t = g.typed(APTPA)
    assert t.n_mids == 20
    assert set(np.unique(t.edge_rel).tolist()) == {_lib.R_AP, _lib.R_PX}


@pytest.mark.skipif(not os.path.exists(REF_GEXF), reason="reference data not present")
def test_streaming_gexf_matches_networkx(dblp_small_tuples):
    g = read_gexf(REF_GEXF)
    assert g.vertices() == dblp_small_tuples[0]
    assert g.edges() == dblp_small_tuples[1]


def _nx_tuples(path):
    import pathsim_oracle as po
    return po.load_gexf_networkx(path)


def test_gexf_roundtrip_synthetic(tmp_path):
    g = synth_dblp(200, 500, 30, seed=4)
    p = tmp_path / "s.gexf"
    write_gexf(g, str(p))
    v, e = _nx_tuples(str(p))
    h = read_gexf(str(p))
    assert h.vertices() == v == g.vertices()
    assert h.edges() == e


def test_gexf_multigraph_and_label_semantics(tmp_path):
    """Parallel edges keep the MultiDiGraph; a repeated (u,v,id) updates in place;
    the XML label attribute overrides the 'label' attvalue; mutual adds both ways."""
    xml = """<?xml version='1.0' encoding='utf-8'?>
<gexf version="1.2" xmlns="http://www.gexf.net/1.2draft">
  <graph defaultedgetype="directed" mode="static">
    <attributes class="edge" mode="static"><attribute id="1" title="label" type="string" /></attributes>
    <attributes class="node" mode="static"><attribute id="0" title="node_type" type="string" /></attributes>
    <nodes>
      <node id="p" label="P"><attvalues><attvalue for="0" value="paper" /></attvalues></node>
      <node id="a" label="A"><attvalues><attvalue for="0" value="author" /></attvalues></node>
      <node id="v" label="V"><attvalues><attvalue for="0" value="venue" /></attvalues></node>
    </nodes>
    <edges>
      <edge id="0" source="a" target="p"><attvalues><attvalue for="1" value="author_of" /></attvalues></edge>
      <edge id="1" source="a" target="p"><attvalues><attvalue for="1" value="author_of" /></attvalues></edge>
      <edge id="1" source="a" target="p"><attvalues><attvalue for="1" value="cites" /></attvalues></edge>
      <edge id="2" source="p" target="v" label="submit_at"><attvalues><attvalue for="1" value="x" /></attvalues></edge>
      <edge id="3" source="v" target="a" type="mutual"><attvalues><attvalue for="1" value="m" /></attvalues></edge>
    </edges>
  </graph>
</gexf>"""
    p = tmp_path / "m.gexf"
    p.write_text(xml)
    v, e = _nx_tuples(str(p))
    h = read_gexf(str(p))
    assert h.vertices() == v
    assert h.edges() == e


def test_gexf_repeated_key_without_label_keeps_label(tmp_path):
    """A repeated (u, v, id) edge without a label updates the edge's data dict
    (networkx ``datadict.update``): the earlier label survives; an edge that
    never gets a label raises KeyError('label') like the reference loop (:123-124)."""
    head = """<?xml version='1.0' encoding='utf-8'?>
<gexf version="1.2" xmlns="http://www.gexf.net/1.2draft">
  <graph defaultedgetype="directed" mode="static">
    <attributes class="edge" mode="static"><attribute id="1" title="label" type="string" />
      <attribute id="2" title="w" type="string" /></attributes>
    <attributes class="node" mode="static"><attribute id="0" title="node_type" type="string" /></attributes>
    <nodes>
      <node id="a" label="A"><attvalues><attvalue for="0" value="author" /></attvalues></node>
      <node id="p" label="P"><attvalues><attvalue for="0" value="paper" /></attvalues></node>
    </nodes>
    <edges>
"""
    tail = "    </edges>\n  </graph>\n</gexf>"
    ok = head + """      <edge id="7" source="a" target="p"><attvalues><attvalue for="1" value="author_of" /></attvalues></edge>
      <edge id="7" source="a" target="p"><attvalues><attvalue for="2" value="x" /></attvalues></edge>
""" + tail
    p = tmp_path / "k.gexf"
    p.write_text(ok)
    v, e = _nx_tuples(str(p))
    h = read_gexf(str(p))
    assert h.edges() == e == [("a", "p", "author_of")]
    bad = head + """      <edge id="7" source="a" target="p"><attvalues><attvalue for="2" value="x" /></attvalues></edge>
""" + tail
    p.write_text(bad)
    with pytest.raises(KeyError):
        _nx_tuples(str(p))
    with pytest.raises(KeyError):
        read_gexf(str(p))


def test_synth_deterministic_and_shaped():
    a = synth_dblp(1000, 3000, 50, seed=9)
    b = synth_dblp(1000, 3000, 50, seed=9)
    assert np.array_equal(a.edge_src, b.edge_src) and np.array_equal(a.edge_dst, b.edge_dst)
    t = a.typed()
    assert (t.n_authors, t.n_papers, t.n_mids) == (1000, 3000, 50)
    ap = t.edge_rel == _lib.R_AP
    # every author writes at least one paper
    assert len(np.unique(t.node_rowid[a.edge_src[ap]])) == 1000


def test_c_abi_rejects_bad_arguments_without_gpu():
    """Argument validation happens host-side before any HIP call."""
    lib = _lib.load()
    rc = lib.dps_cct_topk(None, None, None, None, None, None, None, 10, 5, 300, None, None,
                          None, None, None, 0, 10, None, 10, None, None, None, None, 0, None)
    assert rc == _lib.DPS_ERR_UNSUPPORTED     # tile_w 300 is not a power of two
    assert b"tile_w" in lib.dps_last_error()
    rc = lib.dps_cct_topk(None, None, None, None, None, None, None, 10, 5, 256, None, None,
                          None, None, None, 0, 10, None, 0, None, None, None, None, 0, None)
    assert rc == _lib.DPS_ERR_UNSUPPORTED     # k = 0
    assert lib.dps_csr_build_workspace_size(100, 10) > 0
    # venue skipping: the struct's table width and pointers are validated too
    ws = C.create_string_buffer(1024)
    ws_al = (C.addressof(ws) + 255) // 256 * 256
    vs = _lib.CctExt(1, 1, 1, 65, None, None, None, None)
    rc = lib.dps_cct_topk(8, 8, 8, 8, None, None, None, 10, 5, 256, 8, 8, None, 8,
                          C.addressof(vs), 0, 10, None, 10, 8, 8, 8, ws_al, 512, None)
    assert rc == _lib.DPS_ERR_INVALID and b"n_hv" in lib.dps_last_error()
    vs = _lib.CctExt(1, None, 1, 32, None, None, None, None)
    rc = lib.dps_cct_topk(8, 8, 8, 8, None, None, None, 10, 5, 256, 8, 8, None, 8,
                          C.addressof(vs), 0, 10, None, 10, 8, 8, 8, ws_al, 512, None)
    assert rc == _lib.DPS_ERR_INVALID and b"venue skipping" in lib.dps_last_error()
    # companion u8 tiles belong to tile_w 16384 only
    vs = _lib.CctExt(None, None, None, 0, 8, 8, 8, None)
    rc = lib.dps_cct_topk(8, 8, 8, 8, None, None, None, 10, 5, 256, 8, 8, None, 8,
                          C.addressof(vs), 0, 10, None, 10, 8, 8, 8, ws_al, 512, None)
    assert rc == _lib.DPS_ERR_INVALID and b"16384" in lib.dps_last_error()
    # the T15 widths (7680 / 15360) run without the optimistic passes' tile_sum
    vs = _lib.CctExt(None, None, None, 0, 8, 8, 8, 8)
    rc = lib.dps_cct_topk(8, 8, 8, 8, None, None, None, 10, 5, 15360, 8, 8, None, 8,
                          C.addressof(vs), 0, 10, None, 10, 8, 8, 8, ws_al, 512, None)
    assert rc == _lib.DPS_ERR_UNSUPPORTED and b"15360" in lib.dps_last_error()
    rc = lib.dps_cct_topk(8, 8, 8, 8, None, None, None, 10, 5, 15000, 8, 8, None, 8,
                          None, 0, 10, None, 10, 8, 8, 8, ws_al, 512, None)
    assert rc == _lib.DPS_ERR_UNSUPPORTED and b"15360" in lib.dps_last_error()
    assert lib.dps_heavy_venues(None, 10, 0, None, None) == _lib.DPS_ERR_INVALID
    assert lib.dps_heavy_table(None, None, None, None, 10, None, 65, None, None) == _lib.DPS_ERR_INVALID


def test_tuning_overrides():
    """dps_set_tuning: explicit overrides replace environment variables (the
    default library reads none); bad keys and values are rejected."""
    lib = _lib.load()
    assert lib.dps_get_tuning(_lib.TUNE_WAVES_PER_ROW) == 0
    assert lib.dps_set_tuning(_lib.TUNE_WAVES_PER_ROW, 3) == _lib.DPS_ERR_INVALID
    assert lib.dps_set_tuning(99, 1) == _lib.DPS_ERR_INVALID
    assert lib.dps_set_tuning(_lib.TUNE_TILE_BUILD, 3) == _lib.DPS_ERR_INVALID
    assert lib.dps_set_tuning(_lib.TUNE_BANK_ORDER, 3) == _lib.DPS_ERR_INVALID
    try:
        assert lib.dps_set_tuning(_lib.TUNE_WAVES_PER_ROW, 4) == 0
        assert lib.dps_get_tuning(_lib.TUNE_WAVES_PER_ROW) == 4
    finally:
        lib.dps_set_tuning(_lib.TUNE_WAVES_PER_ROW, 0)
    assert lib.dps_get_tuning(_lib.TUNE_WAVES_PER_ROW) == 0


def test_library_reads_no_environment_knobs():
    """The production library carries no DPATHSIM_* environment names: a stray
    shell variable cannot change what it computes or how fast."""
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"DPATHSIM_" not in data


def _raw_truth(typed):
    """Exact post-distinct sizes from the C oracle (for the bound checks)."""
    import pathsim_oracle as po
    co = po.COracle.from_typed(typed)
    cp, cc, cv, s, g = co.export()
    return cp, cv, s, g, co.diag()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_host_bounds_dominate_device_sizes(seed, dblp_small_tuples):
    """build() sizes every buffer from host_bounds (no device read-back): the
    bounds must dominate nnz(C), sum(C), sum(s) and the bit length of max g."""
    from dpathsim.engine import host_bounds
    graphs = [synth_dblp(3000, 9000, 200, seed=seed),
              synth_dblp(500, 3000, 50, seed=seed, mid_alpha=0.2, authors_lambda=6.0),
              Graph.from_tuples(*dblp_small_tuples)]
    for gr in graphs:
        t = gr.typed()
        b = host_bounds(t)
        cp, cv, s, g, dg = _raw_truth(t)
        assert b.expand >= cp[-1] and b.expand >= int(cv.sum())
        assert b.sum_c >= int(s.sum())
        assert b.key_bits >= max(int(g.max(initial=0)), int(dg.max(initial=0))).bit_length()


def test_cli_arguments():
    from dpathsim.cli import parse
    a = parse(["--synth", "config3", "--all-pairs", "--topk", "10", "--denominator", "diag"])
    assert a.all_pairs and a.denominator == "diag" and a.topk == 10
    a = parse(["--graph", "g.gexf", "--source-name", "Jiawei Han"])
    assert a.source_name == "Jiawei Han" and a.denominator == "rowsum"
    for bad in (["--graph", "g"], ["--graph", "g", "--source-name", "x", "--denominator", "diag"],
                ["--synth", "config3", "--all-pairs", "--topk", "0"],
                ["--graph", "g", "--synth", "config3", "--all-pairs"]):
        with pytest.raises(SystemExit):
            parse(bad)


def test_compat_rejects_a_non_engine_graphframe(tmp_path, dblp_small_tuples):
    """DPathSim_APVPA's second argument replaces the reference's GraphFrame
    (DPathSim_APVPA.py:9); anything but a PathSimEngine (or None) is a TypeError,
    raised before any device work and before the log file is opened."""
    from dpathsim.compat import DPathSim_APVPA
    g = Graph.from_tuples(*dblp_small_tuples)
    log = tmp_path / "run.log"
    with pytest.raises(TypeError, match="PathSimEngine"):
        DPathSim_APVPA(g, object(), "author_0", str(log))
    assert not log.exists()


_NATIVE_CASES = {
    "entities_comments_undirected": """<?xml version='1.0' encoding='utf-8'?>
<!-- a comment before the root -->
<gexf version="1.2" xmlns="http://www.gexf.net/1.2draft" xmlns:viz="http://www.gexf.net/1.2draft/viz">
  <graph defaultedgetype="undirected" mode="static">
    <attributes class="node"><attribute id="t" title="node_type" type="string"/></attributes>
    <attributes class="edge"><attribute id="l" title="label" type="string"/></attributes>
    <nodes>
      <node id="b&amp;1" label="Bee &quot;one&quot; &#233;"><attvalues><attvalue for="t" value="author"/></attvalues><viz:color r="1" g="2" b="3"/></node>
      <node id='a' label='A	tab'><attvalues><attvalue for='t' value='author'/></attvalues></node>
      <node id="p"><attvalues><attvalue for="t" value="paper"/></attvalues></node>
      <node id="a" label="A again"/>
    </nodes>
    <edges>
      <edge id="e1" source="p" target="b&amp;1"><attvalues><attvalue for="l" value="author_of"/></attvalues></edge>
      <edge source="a" target="p" label="author_of"/>
      <edge id="e1" source="b&amp;1" target="p" label="writes"/>
    </edges>
  </graph>
</gexf>""",
    "edge_only_node_typed_later": """<?xml version="1.0"?>
<gexf xmlns="http://www.gexf.net/1.2draft" version="1.2">
  <graph defaultedgetype="directed">
    <attributes class="node"><attribute id="0" title="node_type" type="string"/></attributes>
    <nodes>
      <node id="x" label="X"><attvalues><attvalue for="0" value="venue"/></attvalues></node>
      <node id="y" label="Y"><attvalues><attvalue for="0" value="paper"/></attvalues></node>
    </nodes>
    <edges>
      <edge id="0" source="y" target="x" label="submit_at"/>
      <edge id="1" source="y" target="x" label="submit_at"/>
    </edges>
  </graph>
</gexf>""",
}


@pytest.mark.parametrize("case", sorted(_NATIVE_CASES))
def test_native_gexf_scan_equals_python_loop(tmp_path, case):
    """dps_gexf_open (mmap'ed C++ scanner) and the iterparse loop feed the same
    key collapse / ordering: identical graphs, and both equal networkx's."""
    p = tmp_path / f"{case}.gexf"
    p.write_text(_NATIVE_CASES[case], encoding="utf-8")
    a = read_gexf(str(p), native=True)
    b = read_gexf(str(p), native=False)
    assert a.vertices() == b.vertices() and a.edges() == b.edges()
    assert a.type_names == b.type_names and a.rel_names == b.rel_names
    v, e = _nx_tuples(str(p))
    assert a.vertices() == v and a.edges() == e


def test_native_gexf_declines_latin1(tmp_path):
    """An ISO-8859-1 file with non-ASCII names: the native scanner declines it
    (declared encoding) and the Python loop decodes it as networkx does."""
    text = _NATIVE_CASES["edge_only_node_typed_later"].replace(
        '<?xml version="1.0"?>', '<?xml version="1.0" encoding="ISO-8859-1"?>').replace(
        'label="X"', 'label="J\u00fcrgen M\u00fcller"')
    p = tmp_path / "latin1.gexf"
    p.write_bytes(text.encode("latin-1"))
    with pytest.raises(RuntimeError):
        read_gexf(str(p), native=True)
    a = read_gexf(str(p))
    v, e = _nx_tuples(str(p))
    assert a.vertices() == v and a.edges() == e
    assert "J\u00fcrgen M\u00fcller" in [x[1] for x in a.vertices()]


def test_native_gexf_scan_synthetic_and_fallbacks(tmp_path):
    g = synth_dblp(300, 900, 40, seed=12)
    p = tmp_path / "s.gexf"
    write_gexf(g, str(p))
    a, b = read_gexf(str(p), native=True), read_gexf(str(p), native=False)
    assert a.vertices() == b.vertices() == g.vertices() and a.edges() == b.edges()
    assert np.array_equal(a.edge_src, b.edge_src) and np.array_equal(a.edge_rel_idx, b.edge_rel_idx)
    # outside the native subset: nested <nodes> and numeric attribute types go
    # to the Python loop (which raises / converts as networkx does)
    nested = _NATIVE_CASES["edge_only_node_typed_later"].replace(
        '<node id="y" label="Y">', '<node id="y" label="Y"><nodes><node id="z"/></nodes>')
    p.write_text(nested)
    with pytest.raises(RuntimeError):
        read_gexf(str(p), native=True)
    with pytest.raises(NotImplementedError):
        read_gexf(str(p))
