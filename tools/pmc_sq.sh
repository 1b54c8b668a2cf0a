#!/bin/bash
# SQ/LDS counter passes on the hot kernel (one rocprofv3 run per pass).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  rm -rf gpurun_out/sq_$i
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/sq_$i -o run -- python3 -u tools/hot_once.py \
    > gpurun_out/sq_$i.log 2>&1 || { echo "pass $i failed"; tail -20 gpurun_out/sq_$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob
from collections import defaultdict
tot = defaultdict(float)
for f in glob.glob("gpurun_out/sq_*/**/*counter_collection*.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_cct_topk" in r.get("Kernel_Name", ""):
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(tot): print(f"{k:24s} {tot[k]:.4g}")
PY
