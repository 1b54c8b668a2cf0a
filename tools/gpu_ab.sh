#!/bin/bash
# GPU parity tests, then A/B timing of the current library against ab/libdpathsim_base.so
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python -u tools/ab_hot.py > gpurun_out/ab.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/ab.log; exit 1; }
cat gpurun_out/ab.log
if [ -f ab/libdpathsim_base.so ]; then
  DPATHSIM_LIB=$PWD/ab/libdpathsim_base.so AB_ABLATE= timeout -k 10 300 python -u tools/ab_hot.py > gpurun_out/ab_base.log 2>&1 \
    || { echo "ab base failed"; tail -30 gpurun_out/ab_base.log; exit 1; }
  echo "--- base:"; cat gpurun_out/ab_base.log
fi
