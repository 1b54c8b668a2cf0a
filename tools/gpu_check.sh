#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel stats.
# Every GPU step has its own time limit; the first failure ends the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed: $?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
  || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 > gpurun_out/bench.log 2>&1 \
  || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 \
  || { echo "rocprof failed"; tail -20 gpurun_out/bench_prof.log; exit 1; }
tail -1 gpurun_out/bench_prof.log
find gpurun_out/prof_$TAG -name '*stats*'
