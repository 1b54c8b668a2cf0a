#!/bin/bash
# Round 3 extras on one box: (1) the MFMA heavy-venue probe re-timed in the
# same rocprof profile as the current SIMT kernel (N1); (2) per-shard timing
# for the N = 2/4/8 prediction; (3) configs 4 and 5 through bench.py.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03x}
mkdir -p $O
if [ -z "${SKIP_MFMA:-}" ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mfma_prof -o run -- \
  python3 -u tools/mfma_probe/run_probe.py > $O/mfma_probe.log 2>&1 || { echo "mfma probe failed"; tail -20 $O/mfma_probe.log; exit 1; }
grep -v amdgpu.ids $O/mfma_probe.log | tail -4
fi
if [ -z "${SKIP_SHARD:-}" ]; then
timeout -k 10 300 python3 -u tools/shard_balance.py > $O/shard_balance.txt 2>&1 || { echo "shard balance failed"; tail -20 $O/shard_balance.txt; exit 1; }
grep -v amdgpu.ids $O/shard_balance.txt
fi
if [ -z "${SKIP_CONFIGS:-}" ]; then
for c in config4 config5; do
  timeout -k 10 400 python3 -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$c.log 2>&1 \
    || { echo "bench $c failed"; tail -20 $O/bench_$c.log; exit 1; }
  python3 - <<PY
import json
r = json.loads([l for l in open("$O/bench_$c.log") if l.startswith("{")][-1])
print("$c", "ms/step %.1f" % r["ms_per_step"], "cct %.1f" % r["phases_ms"]["cct_topk"], "value %.3e" % r["value"],
      "frac %.3f" % r["roofline"]["frac"], "venue_skip", r["roofline"]["venue_skip"])
PY
done
fi
