#!/bin/bash
# config4 (APTPA, 200k topics): bench at several tile widths (sparse buckets
# pad to 16 B, so wider tiles mean fewer, fuller buckets).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for W in ${WIDTHS:-8192 16384 32768 65536}; do
  timeout -k 10 300 python -u bench.py --config config4 --tile-w $W --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/bench_c4_w$W.log 2>&1 || { echo "W=$W failed"; tail -20 gpurun_out/bench_c4_w$W.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_c4_w$W.log').read().strip().splitlines()[-1]); print($W, round(d['ms_per_step'],1), d['phases_ms'], '%.3g' % d['value'])"
done
