"""The device-assert debug build (`make debug`: -O1 -g kernels, DPS_DEBUG) gives
the oracle's lists too.  Round 6 found two defects that only the -O1 build
showed -- cross-lane reads under lane-dependent branches (the zero fill, and
the two-register top-k's shift-in) -- so the debug build is a
check of its own: a correct kernel must not depend on the optimiser keeping
values in registers.  One subprocess (the library is chosen when it loads)
runs every case; skipped when the debug library has not been built."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEBUG_LIB = os.path.join(REPO, "distributed-pathsim_amd", "dpathsim", "libdpathsim_debug.so")

SCRIPT = r"""
import sys
import numpy as np
import pathsim_oracle as po
from dpathsim.engine import build_engine
from dpathsim.synth import synth_dblp
from dpathsim import _lib
_lib.load()
print("lib", _lib.LIB_PATH, flush=True)
t = synth_dblp(20000, 60000, 300, seed=5).typed()
co = po.COracle.from_typed(t)
bad = []
for w, k in ((8192, 100), (16384, 100), (16384, 10), (15360, 65), (8192, 10)):
    eng = build_engine(t, tile_w=w)
    got = [a.cpu().numpy() for a in eng.topk(k)]
    want = co.topk(k, 0, t.n_authors)
    n = int(((got[0] != want[0]).any(1) | (got[1] != want[1]).any(1) |
             (got[2].view(np.int64) != want[2].view(np.int64)).any(1)).sum())
    print(f"tile_w {w} k {k}: {n} rows differ", flush=True)
    if n:
        bad.append((w, k, n))
    del eng
print("ok" if not bad else f"mismatch {bad}")
"""


@pytest.mark.skipif(not os.path.exists(DEBUG_LIB), reason="debug library not built (make debug)")
def test_debug_build_matches_oracle():
    env = dict(os.environ, DPATHSIM_LIB=DEBUG_LIB,
               PYTHONPATH=os.pathsep.join([os.path.join(REPO, "distributed-pathsim_amd"),
                                           os.path.join(REPO, "oracle"),
                                           os.environ.get("PYTHONPATH", "")]))
    r = subprocess.run([sys.executable, "-c", SCRIPT], env=env, capture_output=True, text=True,
                       timeout=600)
    out = r.stdout.strip().splitlines()
    assert r.returncode == 0, r.stderr[-2000:]
    assert out and out[0] == f"lib {DEBUG_LIB}", "\n".join(out)
    assert out[-1] == "ok", "\n".join(out)
