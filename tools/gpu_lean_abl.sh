#!/bin/bash
# Lean-kernel variants (ab/libdpathsim_<v>.so for v in $VARIANTS): full config3
# launch time (tools/ab_lean.py, lean mode only) and one rocprofv3 --pmc pass
# each (VALU / SALU / LDS instructions, wave cycles) on the same launch.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
P="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
: > gpurun_out/lean_abl.log
for v in ${VARIANTS}; do
  DPATHSIM_LIB=$PWD/ab/libdpathsim_$v.so AB_MODES=1 AB_REPS=${AB_REPS:-2} timeout -k 10 200 python -u tools/ab_lean.py \
    > gpurun_out/lean_abl_$v.log 2>&1 || { echo "ab $v failed"; tail -20 gpurun_out/lean_abl_$v.log; exit 1; }
  echo "$v: $(grep lean= gpurun_out/lean_abl_$v.log)" | tee -a gpurun_out/lean_abl.log
  if [ "${NO_PMC:-0}" != "1" ]; then
  rm -rf gpurun_out/pmc_$v
  DPATHSIM_LIB=$PWD/ab/libdpathsim_$v.so HOT_ROWS=${HOT_ROWS:-1000000} timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv \
    -d gpurun_out/pmc_$v -o run -- python3 -u tools/hot_once.py > gpurun_out/pmc_$v.log 2>&1 \
    || { echo "pmc $v failed"; tail -20 gpurun_out/pmc_$v.log; exit 1; }
  fi
done
python3 - <<'PY' | tee -a gpurun_out/lean_abl.log
import csv, glob, os
from collections import defaultdict
for d in sorted(glob.glob("gpurun_out/pmc_*/")):
    tot = defaultdict(float)
    for f in glob.glob(d + "**/*counter_collection*.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_cct" in r.get("Kernel_Name", ""):
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
    print(d, " ".join(f"{k}={tot[k]:.4g}" for k in sorted(tot)))
PY
