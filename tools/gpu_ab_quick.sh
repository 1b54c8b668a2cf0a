#!/bin/bash
# Quick A/B: the fast GPU parity tests on the in-tree library, then AB_RUNS
# ("lib:W[:config[:k]]" of ab/*.so) through tools/ab_one.py.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${AB_SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_synth.py tests/test_gpu_edge.py -x -q -s --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_quick.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_quick.log; exit 1; }
tail -2 gpurun_out/pytest_quick.log
fi
: > gpurun_out/ablibs.log
for run in ${AB_RUNS:-}; do
  IFS=: read -r tag W cfg k <<< "$run"
  DPATHSIM_LIB=$PWD/ab/$tag.so AB_TAG=$tag:$W AB_W=$W AB_CONFIG=${cfg:-config3} AB_K=${k:-10} \
    timeout -k 10 300 python -u tools/ab_one.py >> gpurun_out/ablibs.log 2>&1 \
    || { echo "ab $run failed"; tail -20 gpurun_out/ablibs.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/ablibs.log || true
