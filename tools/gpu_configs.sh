#!/bin/bash
# Full-size configs 4 and 5: slice parity vs the C oracle, then one bench line each.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_synth.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "config4 or config5" > gpurun_out/pytest_cfg45.log 2>&1 || { echo "pytest failed: $?"; tail -30 gpurun_out/pytest_cfg45.log; exit 1; }
tail -4 gpurun_out/pytest_cfg45.log
for c in config4 config5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 2 --warmup 1 > gpurun_out/bench_$c.log 2>&1 \
    || { echo "bench $c failed"; tail -20 gpurun_out/bench_$c.log; exit 1; }
  tail -1 gpurun_out/bench_$c.log
done
