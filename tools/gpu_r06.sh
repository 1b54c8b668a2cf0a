#!/bin/bash
# One GPU-box session (round 6).  Sections run when their variable is set:
#   TESTS="<pytest paths/args>"  GPU tests with the in-tree library
#   DEBUG="<pytest paths/args>"  the same with the device-assert debug build
#   BENCH=1                      smoke + bench.py (config3) + rocprofv3 stats of the bench
#   PHASES=1                     profiling build: phase cycles + chunks-per-pass histogram
#   AB=1                         tools/ab_w.py with the in-tree library and every ab/libdpathsim_*.so
# Every GPU step has its own time limit; the first failure ends the script.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06}
mkdir -p $O
LIBDIR=$PWD/distributed-pathsim_amd/dpathsim
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TESTS_LIMIT:-900} python -u -m pytest $TESTS -m gpu -x -v -s --timeout 600 \
    --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed: $?"; tail -40 $O/pytest_gpu.log; exit 1; }
  tail -3 $O/pytest_gpu.log
fi
if [ -n "${DEBUG:-}" ]; then
  DPATHSIM_LIB=$LIBDIR/libdpathsim_debug.so timeout -k 10 ${DEBUG_LIMIT:-700} python -u -m pytest $DEBUG \
    -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_debug.log 2>&1 \
    || { echo "debug pytest failed: $?"; tail -40 $O/pytest_debug.log; exit 1; }
  tail -3 $O/pytest_debug.log
fi
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
    || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
  timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 ${BENCH_ARGS:-} > $O/bench.log 2>&1 \
    || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
  tail -1 $O/bench.log | cut -c1-600
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $O/bench_prof.log 2>&1 \
    || { echo "rocprof failed"; tail -20 $O/bench_prof.log; exit 1; }
  find $O/prof -name '*kernel_stats*' -exec head -4 {} \;
fi
if [ -n "${PHASES:-}" ]; then
  DPATHSIM_LIB=$LIBDIR/libdpathsim_prof.so timeout -k 10 300 \
    python3 -u tools/lean_phases.py > $O/lean_phases.txt 2>&1 || { echo "phases failed"; tail -20 $O/lean_phases.txt; exit 1; }
  grep -v amdgpu.ids $O/lean_phases.txt
fi
if [ -n "${AB:-}" ]; then
  export AB_CASES=${AB_CASES:-16384:1} AB_REPS=${AB_REPS:-3} AB_OPT=${AB_OPT:-0}
  for round in 1 2; do
    timeout -k 10 300 python -u tools/ab_w.py > $O/ab_cur_$round.log 2>&1 || { echo "ab cur failed"; tail -30 $O/ab_cur_$round.log; exit 1; }
    echo "current $round:"; grep -v amdgpu.ids $O/ab_cur_$round.log
    for lib in ab/libdpathsim_*.so; do
      [ -e "$lib" ] || continue
      n=$(basename $lib .so)
      DPATHSIM_LIB=$PWD/$lib timeout -k 10 300 python -u tools/ab_w.py > $O/ab_${n}_$round.log 2>&1 \
        || { echo "ab $n failed"; tail -30 $O/ab_${n}_$round.log; exit 1; }
      echo "$n $round:"; grep -v amdgpu.ids $O/ab_${n}_$round.log
    done
  done
fi
if [ -n "${ROWS:-}" ]; then
  DPATHSIM_LIB=$LIBDIR/libdpathsim_prof.so ROW_OUT=$O/row_times.npz timeout -k 10 300 \
    python3 -u tools/row_times.py > $O/row_times_prof.txt 2>&1 || { echo "row prof failed"; tail -20 $O/row_times_prof.txt; exit 1; }
  grep -v amdgpu.ids $O/row_times_prof.txt
  ROW_PHASE=time ROW_OUT=$O/row_times.npz timeout -k 10 300 \
    python3 -u tools/row_times.py > $O/row_times_ab.txt 2>&1 || { echo "row ab failed"; tail -20 $O/row_times_ab.txt; exit 1; }
  grep -v amdgpu.ids $O/row_times_ab.txt
fi
if [ -n "${REHEARSE:-}" ]; then
  # bench.py --gpus 2 over gloo on this one GPU (the driver's N > 1 runs use
  # RCCL, one GPU per rank) and the C-ABI RCCL gather + known-pattern check
  timeout -k 10 300 python -u -m pytest tests/test_dist.py -m gpu -x -v --timeout 240 \
    --timeout-method thread > $O/pytest_dist.log 2>&1 || { echo "dist tests failed"; tail -30 $O/pytest_dist.log; exit 1; }
  tail -2 $O/pytest_dist.log
  DPATHSIM_BENCH_DEVICE=0 DPATHSIM_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 \
    --steps 2 --warmup 1 > $O/bench_rehearse2.log 2>&1 || { echo "rehearsal failed"; tail -30 $O/bench_rehearse2.log; exit 1; }
  grep '"metric"' $O/bench_rehearse2.log | cut -c1-400
fi
echo "session done"
