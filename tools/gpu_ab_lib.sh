#!/bin/bash
# A/B of the hot kernel across libraries: the current build, then every
# ab/libdpathsim_*.so (tools/ab_w.py; AB_CASES / AB_CONFIG from the environment).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
if [ "${AB_TESTS:-0}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
export AB_CASES=${AB_CASES:-8192:1}
timeout -k 10 300 python -u tools/ab_w.py > gpurun_out/ab_cur.log 2>&1 || { echo "ab cur failed"; tail -30 gpurun_out/ab_cur.log; exit 1; }
echo "current:"; grep -v amdgpu.ids gpurun_out/ab_cur.log
for lib in ab/libdpathsim_*.so; do
  n=$(basename $lib .so)
  DPATHSIM_LIB=$PWD/$lib timeout -k 10 300 python -u tools/ab_w.py > gpurun_out/ab_$n.log 2>&1 || { echo "ab $n failed"; tail -30 gpurun_out/ab_$n.log; exit 1; }
  echo "$n:"; grep -v amdgpu.ids gpurun_out/ab_$n.log
done
