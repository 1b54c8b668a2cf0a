#!/bin/bash
# Global-atomic tile build (config4): many-mid tests, config4 slices, build phases.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_synth.py tests/test_gpu_fullsize.py -m gpu -x -v \
  --timeout 500 --timeout-method thread -k "many_mids or config4" > gpurun_out/pytest_c4_tiles.log 2>&1 \
  || { echo "pytest failed"; tail -40 gpurun_out/pytest_c4_tiles.log; exit 1; }
tail -2 gpurun_out/pytest_c4_tiles.log
AB_CONFIG=config4 AB_REPS=5 timeout -k 10 300 python -u tools/build_ab.py > gpurun_out/build_ab_c4_tiles.log 2>&1 \
  || { echo "build_ab failed"; tail -20 gpurun_out/build_ab_c4_tiles.log; exit 1; }
grep phase gpurun_out/build_ab_c4_tiles.log
