#!/bin/bash
# Round 5: boundary + optimistic-pass GPU tests, then the hot kernel A/B with
# and without the optimistic 4-bit passes (judged in the epilogue) on config3.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-r05c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_boundary.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for opt in 0 1 0 1; do
  AB_OPT=$opt AB_CASES=16384:1 AB_REPS=3 timeout -k 10 200 python -u tools/ab_w.py > $O/ab_opt$opt.log 2>&1 \
    || { echo "ab failed"; tail -20 $O/ab_opt$opt.log; exit 1; }
  echo "opt=$opt: $(grep 'W=16384' $O/ab_opt$opt.log)"
done
