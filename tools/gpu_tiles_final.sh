#!/bin/bash
# Tile-build change check: GPU test suite, then config3 / config5 build phases.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_tiles_final.log 2>&1 \
  || { echo "pytest failed"; tail -30 gpurun_out/pytest_tiles_final.log; exit 1; }
tail -1 gpurun_out/pytest_tiles_final.log
for c in config3 config5; do
  AB_CONFIG=$c AB_REPS=7 timeout -k 10 300 python -u tools/build_ab.py > gpurun_out/build_ab_tf_$c.log 2>&1 \
    || { echo "build_ab $c failed"; tail -20 gpurun_out/build_ab_tf_$c.log; exit 1; }
  grep phase gpurun_out/build_ab_tf_$c.log
done
