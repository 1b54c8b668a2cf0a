#!/bin/bash
# Round 3: configs 4 and 5 at both tile formats, venue skipping on / off
# (bench.py, 3 steps each) -- which default fits which shape.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03c45}
mkdir -p $O
for run in ${RUNS:-config4:8192:0 config4:16384:0 config5:8192:0 config5:16384:0}; do
  IFS=: read c w vs <<< "$run"
  timeout -k 10 400 python3 -u bench.py --config $c --tile-w $w --venue-skip $vs --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_${c}_${w}_$vs.log 2>&1 \
    || { echo "bench $run failed"; tail -20 $O/bench_${c}_${w}_$vs.log; exit 1; }
  python3 - <<PY
import json
r = json.loads([l for l in open("$O/bench_${c}_${w}_$vs.log") if l.startswith("{")][-1])
rf = r["roofline"]
print("$run", "ms/step %.1f" % r["ms_per_step"], "cct %.1f" % r["phases_ms"]["cct_topk"], "value %.3e" % r["value"],
      "frac %.3f" % rf["frac"], "passes", rf["executed"]["passes"], "chunks", rf["executed"]["chunks"], flush=True)
PY
done
