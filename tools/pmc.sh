#!/bin/bash
# HBM traffic of the hot kernel from PMC counters (MI355X_MICROARCH.md, HBM/rocprofv3):
# FETCH_SIZE and WRITE_SIZE in separate passes, then tools/pmc_summary.py applies the
# gfx950 corrections and writes gpurun_out/pmc_hot.json.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
CMD="python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline"
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmc_$c
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_$c -o run -- $CMD \
    > gpurun_out/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -20 gpurun_out/pmc_$c.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE gpurun_out/pmc_hot.json
