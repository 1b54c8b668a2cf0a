#!/bin/bash
# Round 5, first call: baseline bench on this box, then a PC-sampling attempt
# on the hot kernel (config3, first HOT_ROWS rows) to see where its cycles go.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r05a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.log 2>&1 \
  || { echo "bench failed"; tail -30 $O/bench.log; exit 1; }
grep '"metric"' $O/bench.log | cut -c1-300
timeout -s KILL 60 rocprofv3 -L > $O/list.txt 2>&1 || echo "list rc $?"
grep -i -A12 "pc.sampl" $O/list.txt | head -60
HOT_ROWS=${HOT_ROWS:-300000} timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled \
  --pc-sampling-method ${PCM:-stochastic} --pc-sampling-unit ${PCU:-cycles} \
  --pc-sampling-interval ${PCI:-262144} --output-format csv -d $O/pcs -o run -- \
  python3 -u tools/hot_once.py > $O/pcs.log 2>&1 || { echo "pcs rc $?"; tail -20 $O/pcs.log; exit 1; }
tail -3 $O/pcs.log
find $O/pcs -type f | xargs ls -la
