#!/bin/bash
# Round 3: venue skipping on the dual-format W = 16384 kernel -- parity, then A/B.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-r03d}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_venue_skip.py tests/test_gpu_counters.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed: $?"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for VS in 1 0; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --venue-skip $VS > $O/bench_vs$VS.log 2>&1 \
    || { echo "bench vs=$VS failed"; tail -20 $O/bench_vs$VS.log; exit 1; }
done
python - <<PY
import json
for VS in (1, 0):
    r = json.loads(open(f"$O/bench_vs{VS}.log").read().strip().splitlines()[-1])
    rf = r["roofline"]
    print("venue_skip", VS, "ms/step %.2f" % r["ms_per_step"], "cct %.2f" % r["phases_ms"]["cct_topk"],
          "passes", rf["passes"], "chunks", rf["chunks"], "verified", rf["verified"], "value %.3e" % r["value"])
PY
