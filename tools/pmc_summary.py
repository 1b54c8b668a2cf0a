"""Per-launch HBM bytes of the hot kernel from rocprofv3 --pmc CSVs.

traffic = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 per dispatch of k_cct_topk:
FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of
wide (16 B/lane) coalesced reads, which is how the kernel reads its C^T chunks
(MI355X_MICROARCH.md, section HBM).
usage: pmc_summary.py FETCH_DIR WRITE_DIR OUT_JSON
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_dispatch(d, counter, kernel="k_cct_topk"):
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection csv under {d}")
    vals = defaultdict(float)
    for f in files:
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            if kernel in name and row.get("Counter_Name") == counter:
                vals[row.get("Dispatch_Id") or row.get("Correlation_Id")] += float(row["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel} in {d}")
    return sorted(vals.values())


fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
write = per_dispatch(sys.argv[2], "WRITE_SIZE")
f_kib = sum(fetch) / len(fetch)
w_kib = sum(write) / len(write)
rec = {"kernel": "k_cct_topk", "config": "config3", "world": 1,
       "tile_w": int(sys.argv[4]) if len(sys.argv) > 4 else 8192,
       "fetch_size_kib": f_kib, "write_size_kib": w_kib,
       "hbm_bytes_per_launch": 2 * f_kib * 1024 + w_kib * 1024,
       "rule": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950: FETCH_SIZE = half of 16-B/lane reads)",
       "dispatches": [len(fetch), len(write)]}
json.dump(rec, open(sys.argv[3], "w"), indent=1)
print(json.dumps(rec))
