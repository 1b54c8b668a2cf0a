"""Drive tools/mfma_probe/probe.hip on a config's heavy-venue panel (research;
PROBE_CONFIG, default config3; config5 for the round-5 A/B at BASELINE
config 5's shape, PROBE_K the list of panel widths).

Builds the engine, takes the K venues with the most authors (largest n_v, so
largest n_v^2), lays C[y, v] (v heavy, clamped to 127) out as a dense i8 panel
in target-label order, checks one 128x256 block of the MFMA product against
torch, then times the full 1M x 1M heavy product with the epilogue stand-in,
for K in 32, 64, 128, at two threshold settings (none pass / the rows' k-th
counts).  Prints JSON lines.
"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "distributed-pathsim_amd"))
import numpy as np
import torch

from dpathsim.engine import build_engine
from dpathsim.synth import synth_config

lib = ctypes.CDLL(os.path.join(HERE, "libmfmaprobe.so"))
lib.probe_run.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                          ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
from dpathsim.synth import CONFIGS
cfg = os.environ.get("PROBE_CONFIG", "config3")
kk = CONFIGS[cfg][4]
t = synth_config(cfg).typed()
eng = build_engine(t)
NA, NV = t.n_authors, t.n_mids
nnz = eng.info.nnz_c
dev = eng.device
c_ptr = eng.tensor("c_ptr")[: NA + 1]
col = eng.tensor("c_col")[:nnz].long()
val = eng.tensor("c_val")[:nnz]
rank = eng.tensor("t_rank")[:NA].long()
row = torch.repeat_interleave(torch.arange(NA, device=dev), c_ptr[1:] - c_ptr[:-1])
n_v = torch.bincount(col, minlength=NV)
idx, cnt, sc = eng.topk(kk)
torch.cuda.synchronize()
# the SIMT hot kernel itself, timed in the same process (and rocprof profile)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
eng.topk(kk)
e1.record()
torch.cuda.synchronize()
print(json.dumps({"config": cfg, "k": kk, "simt_topk_ms": e0.elapsed_time(e1),
                  "n_authors": NA, "n_mids": NV}), flush=True)
kth_m = cnt[:, -1].to(torch.int32)          # the k-th entry's count per row (original order)
thr_real = torch.empty(NA, dtype=torch.int32, device=dev)
thr_real[rank] = torch.clamp(kth_m, min=1)
res = []
for K in [int(v) for v in os.environ.get("PROBE_K", "32,64,128").split(",")]:
    heavy = torch.argsort(n_v, descending=True)[:K]
    hmap = torch.full((NV,), -1, dtype=torch.long, device=dev)
    hmap[heavy] = torch.arange(K, device=dev)
    share = float((n_v[heavy].double() ** 2).sum() / (n_v.double() ** 2).sum())
    sel = hmap[col] >= 0
    panel = torch.zeros((NA, K), dtype=torch.int8, device=dev)
    panel[rank[row[sel]], hmap[col[sel]]] = torch.clamp(val[sel], max=127).to(torch.int8)
    counter = torch.zeros(1, dtype=torch.int64, device=dev)
    dump = torch.zeros((128, 256), dtype=torch.int32, device=dev)
    thr_none = torch.full((NA,), 2 ** 30, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    rc = lib.probe_run(panel.data_ptr(), NA, K, thr_none.data_ptr(), 256, counter.data_ptr(),
                       dump.data_ptr(), st)
    torch.cuda.synchronize()
    full = (panel[:128].double() @ panel[:256].double().T).to(torch.int32)
    # the dump holds the first B set of waves 0 and 1: sources 0-31 and 64-95
    want = torch.zeros_like(dump)
    want[0:32], want[64:96] = full[0:32], full[64:96]
    ok = bool(torch.equal(dump, want))
    out = {"config": cfg, "K": K, "heavy_share_of_terms": share, "verify_block_exact": ok,
           "rc": rc}
    for name, thr in (("no_candidates", thr_none), ("kth_count_threshold", thr_real)):
        counter.zero_()
        lib.probe_run(panel.data_ptr(), NA, K, thr.data_ptr(), NA, counter.data_ptr(), None, st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        counter.zero_()
        e0.record()
        lib.probe_run(panel.data_ptr(), NA, K, thr.data_ptr(), NA, counter.data_ptr(), None, st)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        out[name] = {"ms": ms, "blocks_passing": int(counter.item()),
                     "int8_tops": 2.0 * NA * NA * K / (ms * 1e-3) / 1e12}
    print(json.dumps(out), flush=True)
    del panel
