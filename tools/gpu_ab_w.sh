#!/bin/bash
# Hot-kernel A/B (tools/ab_w.py) across tile widths / tile orders, optionally after the GPU tests.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
if [ "${AB_TESTS:-1}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
timeout -k 10 400 python -u tools/ab_w.py > gpurun_out/ab_w.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/ab_w.log; exit 1; }
cat gpurun_out/ab_w.log
