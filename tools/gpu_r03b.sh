#!/bin/bash
# Round 3: 4-bit-counter tiles (W = 16384) -- parity on the fast GPU tests, then
# the bench at W = 16384 (new default) against W = 8192.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-r03b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_synth.py tests/test_gpu_counters.py tests/test_gpu_edge.py \
  tests/test_gpu_parity.py tests/test_gpu_venue_skip.py tests/test_gpu_cli.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed: $?"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for W in 16384 8192; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --tile-w $W > $O/bench_w$W.log 2>&1 \
    || { echo "bench W=$W failed"; tail -20 $O/bench_w$W.log; exit 1; }
done
python - <<PY
import json
for W in (16384, 8192):
    r = json.loads(open(f"$O/bench_w{W}.log").read().strip().splitlines()[-1])
    rf = r["roofline"]
    print(W, "ms/step %.2f" % r["ms_per_step"], "cct %.2f" % r["phases_ms"]["cct_topk"],
          "passes", rf["passes"], "chunks", rf["chunks"], "floor %.1f ms" % rf["lds_floor_ms"],
          "frac %.3f" % rf["frac"], "value %.3e" % r["value"])
PY
