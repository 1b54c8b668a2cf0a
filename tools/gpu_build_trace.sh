#!/bin/bash
# Kernel traces of one device build (tools/build_trace.py) on config3 and config4.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${TAG:-btrace}
mkdir -p $O
for cfg in config3:16384 config4:8192; do
  c=${cfg%:*}
  AB_CONFIG=$c AB_W=${cfg#*:} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$c -o run -- \
    python3 -u tools/build_trace.py > $O/$c.log 2>&1 || { echo "trace $c failed"; tail -20 $O/$c.log; exit 1; }
  python3 tools/build_trace_summary.py $(find $O/$c -name '*kernel_trace.csv' | head -1) > $O/${c}_build.txt
  tail -1 $O/${c}_build.txt
done
