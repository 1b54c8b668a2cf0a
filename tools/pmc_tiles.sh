#!/bin/bash
# PMC counters of the device build's kernels (tools/build_ab.py, one setting,
# one timed build): three --pmc passes, each in its own rocprofv3 run, summed per
# kernel -> gpurun_out/pmc_tiles.txt.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i + 1))
  rm -rf gpurun_out/pmc_tiles_$i
  AB_REPS=1 AB_ENV="${AB_ENV:-X=1}" timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv \
    -d gpurun_out/pmc_tiles_$i -o run -- python3 -u tools/build_ab.py > gpurun_out/pmc_tiles_$i.log 2>&1 \
    || { echo "pmc pass $i failed"; tail -20 gpurun_out/pmc_tiles_$i.log; exit 1; }
done
python3 - <<'PY' | tee gpurun_out/pmc_tiles.txt
import csv, glob
from collections import defaultdict
tot = defaultdict(lambda: defaultdict(float))
calls = defaultdict(set)
for f in glob.glob("gpurun_out/pmc_tiles_*/**/*counter_collection*.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].split("::")[-1][:32]
        tot[n][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[(n, r["Counter_Name"])].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
for n, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:14]:
    k = max(len(calls[(n, "SQ_WAVES")]), 1)
    print(n, f"(x{k} dispatches, per dispatch:)")
    print("   " + "  ".join(f"{cn}={v / max(len(calls[(n, cn)]), 1):.4g}" for cn, v in sorted(c.items())))
PY
