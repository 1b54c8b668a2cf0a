#!/bin/bash
# SQ_INSTS_VALU/SALU/LDS of the hot kernel under each DPATHSIM_ABLATE value in $ABL
# (one rocprofv3 --pmc pass per value), then the per-row counters (ablate 8).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
P="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES"
for a in ${ABL:-0 2 4}; do
  rm -rf gpurun_out/valu_$a
  DPATHSIM_ABLATE=$a timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/valu_$a -o run -- python3 -u tools/hot_once.py \
    > gpurun_out/valu_$a.log 2>&1 || { echo "pass $a failed"; tail -20 gpurun_out/valu_$a.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, os
from collections import defaultdict
for d in sorted(glob.glob("gpurun_out/valu_*/")):
    tot = defaultdict(float)
    for f in glob.glob(d + "**/*counter_collection*.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_cct_topk" in r.get("Kernel_Name", ""):
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
    print(d, " ".join(f"{k}={tot[k]:.4g}" for k in sorted(tot)))
PY
DPATHSIM_LIB=$PWD/distributed-pathsim_amd/dpathsim/libdpathsim_prof.so timeout -k 10 120 python3 -u tools/ab_hot.py > gpurun_out/cnt.log 2>&1 || { echo "counters failed"; tail -5 gpurun_out/cnt.log; exit 1; }
grep counters gpurun_out/cnt.log
