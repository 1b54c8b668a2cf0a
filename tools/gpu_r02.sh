#!/bin/bash
# One GPU-box session (round 2): parity tests, smoke, bench, rocprof kernel
# stats, counter list, PMC passes.  Every GPU step has its own time limit; the
# first failure ends the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 900 --timeout-method thread \
  ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed: $?"; tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_$TAG.log
fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
  || { echo "smoke failed"; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench_$TAG.log 2>&1 \
  || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof_$TAG.log 2>&1 \
  || { echo "rocprof failed"; tail -20 gpurun_out/bench_prof_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_prof_$TAG.log
find gpurun_out/prof_$TAG -name '*stats*'
if [ -n "${PMC:-}" ]; then
  timeout -k 5 60 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || echo "counter list failed (ignored)"
  tools/pmc_hot.sh || exit 1
fi
