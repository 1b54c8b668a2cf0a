#!/bin/bash
# Round 5: the boundary GPU tests (ADVICE r04 / VERDICT r04 #6), then PMC
# passes for the instruction cache and instruction mix of the hot kernel.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r05b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_boundary.py tests/test_dist.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
export HOT_ROWS=1000000
declare -A PASS
PASS[ic1]="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE GRBM_GUI_ACTIVE"
PASS[ic2]="SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
PASS[mix]="SQ_INSTS_LDS_ATOMIC SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES"
for p in ic1 ic2 mix; do
  timeout -s KILL 90 rocprofv3 --pmc ${PASS[$p]} --output-format csv -d $O/pmc_$p -o run -- \
    python3 -u tools/hot_once.py > $O/pmc_$p.log 2>&1 \
    || { echo "pmc pass $p failed"; tail -20 $O/pmc_$p.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for p in ("ic1", "ic2", "mix"):
    tot = collections.defaultdict(float)
    for f in glob.glob(f"gpurun_out/r05b/pmc_{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_cct1" in r.get("Kernel_Name", ""):
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
    print(p, {k: f"{v:.4g}" for k, v in tot.items()})
PY
