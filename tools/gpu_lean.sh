#!/bin/bash
# Lean-kernel check: quick GPU parity tests (lean kernel is the default at
# W = 8192), then the A/B against the general kernel on config3 (and AB2_CONFIG).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-lean}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_synth.py tests/test_gpu_edge.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
fi
timeout -k 10 300 python -u tools/ab_lean.py > gpurun_out/ab_$TAG.log 2>&1 || { echo "ab failed"; tail -20 gpurun_out/ab_$TAG.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_$TAG.log
if [ -n "${AB2_CONFIG:-}" ]; then
AB_CONFIG=$AB2_CONFIG AB_K=${AB2_K:-10} timeout -k 10 400 python -u tools/ab_lean.py > gpurun_out/ab2_$TAG.log 2>&1 || { echo "ab2 failed"; tail -20 gpurun_out/ab2_$TAG.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab2_$TAG.log
fi
