#!/bin/bash
# rocprofv3 --pmc passes (stall / issue breakdown) of the hot kernel for lean
# variants ab/libdpathsim_<v>.so on the full config3 launch (tools/hot_once.py).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
PA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
PB="SQ_INSTS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INSTS_VALU"
PD="SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INST_LEVEL_LDS SQ_WAVE_CYCLES"
PC="SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES"
for v in ${VARIANTS}; do
  for pass in ${PASSES:-A B C}; do
    eval P=\$P$pass
    rm -rf gpurun_out/pmc2_${v}_$pass
    DPATHSIM_LIB=$PWD/ab/libdpathsim_$v.so HOT_ROWS=${HOT_ROWS:-1000000} timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv \
      -d gpurun_out/pmc2_${v}_$pass -o run -- python3 -u tools/hot_once.py > gpurun_out/pmc2_${v}_$pass.log 2>&1 \
      || { echo "pmc $v $pass failed"; tail -20 gpurun_out/pmc2_${v}_$pass.log; exit 1; }
  done
done
python3 - <<'PY' | tee gpurun_out/lean_pmc.txt
import csv, glob, os, re
from collections import defaultdict
res = defaultdict(lambda: defaultdict(float))
for d in sorted(glob.glob("gpurun_out/pmc2_*_?/")):
    v = re.match(r"gpurun_out/pmc2_(.*)_[A-D]/", d).group(1)
    for f in glob.glob(d + "**/*counter_collection*.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_cct" in r.get("Kernel_Name", ""):
                res[v][r["Counter_Name"]] += float(r["Counter_Value"])
for v, t in res.items():
    print(v, " ".join(f"{k}={t[k]:.4g}" for k in sorted(t)))
PY
