"""Bytes and build milliseconds of the hot kernel's operand sets (C^T tiles,
companion u8 half tiles, heavy-venue table) for a config at the engine
defaults: the cost side of ADVICE r03's 'build the half tiles only when
needed'.  Prints one JSON line per config.
  python tools/tile_mem.py config3 config5"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-pathsim_amd"))
import torch  # noqa: E402

import dpathsim  # noqa: E402
from dpathsim.engine import PathSimEngine  # noqa: E402
from dpathsim.synth import CONFIGS, synth_config  # noqa: E402

for cfg in sys.argv[1:] or ["config3"]:
    t = synth_config(cfg).typed(dpathsim.METAPATHS[CONFIGS[cfg][3]])
    eng = PathSimEngine(t)
    eng.upload().build()
    eng.build(timed=True)
    d = eng._dev
    used = lambda off: int(d[off][-1].item()) * 4 if d.get(off) is not None else 0   # noqa: E731
    rec = {"config": cfg, "tile_w": eng.tile_w, "nnz_C": eng.info.nnz_c,
           "tile_ent_bytes": used("tile_off"),
           "half_ent_bytes": used("half_off"),
           "tile_off_bytes": d["tile_off"].numel() * 4 * 2,          # tile_off + tile_maxc
           "half_off_bytes": (d["half_off"].numel() * 4 * 2) if d.get("half_off") is not None else 0,
           "hv_c_bytes": d["hv_c"].numel() * 2 if d.get("hv_c") is not None else 0,
           "phase_ms": {k: round(v, 3) for k, v in eng.info.phase_ms.items() if k != "host_total"}}
    print(json.dumps(rec), flush=True)
    del eng
    torch.cuda.empty_cache()
