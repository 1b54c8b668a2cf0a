#!/bin/bash
# PMC counters of the hot kernel at HEAD on the bench launch (config3, all 1M
# rows, tile_w $HOT_W (default 16384), k 10), one rocprofv3 --pmc pass per counter group
# (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE in separate passes; <= 8 SQ
# counters per pass), then tools/pmc_hot_summary.py -> gpurun_out/pmc_hot.json.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
export HOT_ROWS=${HOT_ROWS:-1000000}
export HOT_W=${HOT_W:-16384}
declare -A PASS
PASS[fetch]="FETCH_SIZE"
PASS[write]="WRITE_SIZE"
PASS[valu]="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
PASS[lds]="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
for p in ${PASSES:-fetch write valu lds}; do
  rm -rf gpurun_out/pmc_$p
  timeout -s KILL 150 rocprofv3 --pmc ${PASS[$p]} --output-format csv -d gpurun_out/pmc_$p -o run -- \
    python3 -u tools/hot_once.py > gpurun_out/pmc_$p.log 2>&1 \
    || { echo "pmc pass $p failed"; tail -20 gpurun_out/pmc_$p.log; exit 1; }
done
python3 tools/pmc_hot_summary.py gpurun_out gpurun_out/pmc_hot.json
