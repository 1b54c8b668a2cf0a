#!/bin/bash
# One GPU-box session (round 5): all GPU parity tests, smoke, bench, rocprof
# kernel stats, and (PMC=1) the hot kernel's PMC passes.  Every GPU step has
# its own time limit; the first failure ends the script.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${TAG:-r05s}
O=gpurun_out/$TAG
mkdir -p $O
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 900 --timeout-method thread \
  ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1 || { echo "pytest failed: $?"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > $O/bench.log 2>&1 \
  || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_prof.log 2>&1 \
  || { echo "rocprof failed"; tail -20 $O/bench_prof.log; exit 1; }
tail -1 $O/bench_prof.log
find $O/prof -name '*stats*'
if [ -n "${PMC:-}" ]; then
  tools/pmc_hot.sh || exit 1
  mv gpurun_out/pmc_hot.json $O/ && mkdir -p $O/pmc && mv gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_valu gpurun_out/pmc_lds $O/pmc/
fi
if [ -n "${SHARD:-}" ]; then
  timeout -k 10 300 python3 -u tools/shard_balance.py > $O/shard_balance.txt 2>&1 \
    || { echo "shard_balance failed"; tail -20 $O/shard_balance.txt; exit 1; }
  grep -v amdgpu.ids $O/shard_balance.txt
fi
if [ -n "${PHASES:-}" ]; then
  DPATHSIM_LIB=$PWD/distributed-pathsim_amd/dpathsim/libdpathsim_prof.so timeout -k 10 300 \
    python3 -u tools/lean_phases.py > $O/lean_phases.txt 2>&1 || { echo "phases failed"; tail -20 $O/lean_phases.txt; exit 1; }
  cat $O/lean_phases.txt
fi
if [ -n "${AB:-}" ]; then
  export AB_CASES=${AB_CASES:-16384:1} AB_REPS=${AB_REPS:-3}
  timeout -k 10 300 python -u tools/ab_w.py > $O/ab_cur.log 2>&1 || { echo "ab cur failed"; tail -30 $O/ab_cur.log; exit 1; }
  echo "current:"; grep -v amdgpu.ids $O/ab_cur.log
  for lib in ab/libdpathsim_*.so; do
    n=$(basename $lib .so)
    DPATHSIM_LIB=$PWD/$lib timeout -k 10 300 python -u tools/ab_w.py > $O/ab_$n.log 2>&1 || { echo "ab $n failed"; tail -30 $O/ab_$n.log; exit 1; }
    echo "$n:"; grep -v amdgpu.ids $O/ab_$n.log
  done
fi
