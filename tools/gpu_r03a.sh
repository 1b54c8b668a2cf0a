#!/bin/bash
# Round 3, first GPU session: venue-skipping parity + A/B bench on config3.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r03a
export TMPDIR=/tmp
O=gpurun_out/r03a
timeout -k 10 600 python -u -m pytest tests/test_gpu_venue_skip.py tests/test_gpu_synth.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed: $?"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_vs.log 2>&1 \
  || { echo "bench failed"; tail -20 $O/bench_vs.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-venue-skip > $O/bench_novs.log 2>&1 \
  || { echo "bench failed"; tail -20 $O/bench_novs.log; exit 1; }
python - <<'PY'
import json
for n in ("bench_vs", "bench_novs"):
    r = json.loads(open(f"gpurun_out/r03a/{n}.log").read().strip().splitlines()[-1])
    print(n, "ms/step %.2f" % r["ms_per_step"], "cct %.2f" % r["phases_ms"]["cct_topk"],
          "passes", r["roofline"]["passes"], "chunks", r["roofline"]["chunks"], "value %.3e" % r["value"])
PY
