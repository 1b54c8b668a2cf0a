#!/bin/bash
# Profiling build of the hot kernel on config3 rows [0, 200k) at W = 8192:
# timings under the ablations (1 no LDS adds, 2 no scoring, 4 no scatter),
# event counters (8) and shader-clock phase cycles (16); then SQ_INSTS_VALU per
# ablation (one --pmc pass each).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
export DPATHSIM_LIB=$PWD/distributed-pathsim_amd/dpathsim/libdpathsim_prof.so
AB_W=8192 AB_ABLATE="${ABL_T:-1,2,4,32,64,16}" timeout -k 10 300 python3 -u tools/ab_hot.py > gpurun_out/ab_hot.log 2>&1 \
  || { echo "ab_hot failed"; tail -20 gpurun_out/ab_hot.log; exit 1; }
cat gpurun_out/ab_hot.log
P="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
for a in ${ABL_P:-0 1 2 4 32 64}; do
  rm -rf gpurun_out/valu_$a
  DPATHSIM_ABLATE=$a HOT_ROWS=200000 timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/valu_$a -o run -- python3 -u tools/hot_once.py \
    > gpurun_out/valu_$a.log 2>&1 || { echo "pass $a failed"; tail -20 gpurun_out/valu_$a.log; exit 1; }
done
python3 - <<'PY'
import csv, glob
from collections import defaultdict
for d in sorted(glob.glob("gpurun_out/valu_*/")):
    tot = defaultdict(float)
    for f in glob.glob(d + "**/*counter_collection*.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_cct_topk" in r.get("Kernel_Name", ""):
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
    print(d, " ".join(f"{k}={tot[k]:.4g}" for k in sorted(tot)))
PY
