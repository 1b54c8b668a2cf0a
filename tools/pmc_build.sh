#!/bin/bash
# SQ counters of every kernel of one config3 step (build kernels included):
# where the build's time goes (waiting vs issuing).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
P="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD"
rm -rf gpurun_out/pmc_build
timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pmc_build -o run -- \
  python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_build.log 2>&1 \
  || { echo "pmc failed"; tail -20 gpurun_out/pmc_build.log; exit 1; }
python3 - <<'PY'
import csv, glob
from collections import defaultdict
tot = defaultdict(lambda: defaultdict(float))
for f in glob.glob("gpurun_out/pmc_build/**/*counter_collection*.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].split("::")[-1][:40]
        tot[n][r["Counter_Name"]] += float(r["Counter_Value"])
for n, c in sorted(tot.items(), key=lambda kv: -kv[1]["SQ_WAVE_CYCLES"])[:20]:
    w = c["SQ_WAVE_CYCLES"] or 1
    print(f"{n:40s} waves {c['SQ_WAVES']:9.0f} wcyc {w:10.3g} wait {c['SQ_WAIT_ANY']/w:5.2f} "
          f"stall {c['SQ_WAIT_INST_ANY']/w:5.2f} active {c['SQ_ACTIVE_INST_ANY']/w:5.2f} "
          f"valu {c['SQ_INSTS_VALU']:9.3g} lds {c['SQ_INSTS_LDS']:9.3g} vmem {c['SQ_INSTS_VMEM_RD']:9.3g}")
PY
