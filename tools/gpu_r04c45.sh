#!/bin/bash
# Round 4: configs 4 and 5 at the engine defaults (bench.py --config, 3 steps),
# plus one timed build per config (phase split).
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04c45}
mkdir -p $O
for c in ${CONFIGS:-config4 config5}; do
  timeout -k 10 500 python3 -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$c.log 2>&1 \
    || { echo "bench $c failed"; tail -20 $O/bench_$c.log; exit 1; }
  python3 - <<PY
import json
r = json.loads([l for l in open("$O/bench_$c.log") if l.startswith("{")][-1])
rf = r["roofline"]
print("$c", "ms/step %.1f" % r["ms_per_step"], "cct %.1f" % r["phases_ms"]["cct_topk"], "value %.3e" % r["value"],
      "frac %.3f" % rf["frac"], "passes", rf["executed"]["passes"], "chunks", rf["executed"]["chunks"],
      "spgemm frac %.3f" % r["spgemm_roofline"]["frac"], "tile_w", r["config"]["tile_w"], flush=True)
PY
done
