#!/bin/bash
# Round 5: configs 4 and 5 at the engine defaults (bench.py --config, 3 steps),
# plus one timed build per config (phase split).
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05c45}
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
if [ -n "${MFMA:-}" ]; then
  # MFMA-vs-SIMT A/B at BASELINE config 5's shape: the probe's heavy-venue
  # panel product and the SIMT hot kernel (k = 100) in the same rocprof profile
  [ -f tools/mfma_probe/libmfmaprobe.so ] || { echo "probe library missing"; exit 1; }
  PROBE_CONFIG=config5 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mfma5 -o run -- \
    python3 -u tools/mfma_probe/run_probe.py > $O/mfma5.log 2>&1 || { echo "probe failed"; tail -20 $O/mfma5.log; exit 1; }
  grep '^{' $O/mfma5.log
  find $O/mfma5 -name '*kernel_stats.csv' -exec head -6 {} \;
fi
