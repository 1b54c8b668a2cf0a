#!/bin/bash
# Build-path iteration on the GPU box: quick parity (tile build consumers),
# then the build phase A/B (tools/build_ab.py) and a rocprof of the build.
# Every GPU step has its own time limit; the first failure ends the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-build}
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_counters.py tests/test_gpu_parity.py tests/test_gpu_synth.py ${PYTEST_EXTRA:-} \
  > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed: $?"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -n 2 gpurun_out/pytest_$TAG.log
AB_ENV="${AB_ENV:-DPATHSIM_TILE_LPB=4096}" timeout -k 10 300 python -u tools/build_ab.py \
  > gpurun_out/build_ab_$TAG.log 2>&1 || { echo "build_ab failed"; tail -20 gpurun_out/build_ab_$TAG.log; exit 1; }
cat gpurun_out/build_ab_$TAG.log | grep env
timeout -k 10 300 tools/prof_build.sh > /dev/null 2>&1 || { echo "prof_build failed"; exit 1; }
head -n 25 gpurun_out/prof_build_summary.txt
