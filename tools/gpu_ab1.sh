#!/bin/bash
# Round 5: hot kernel A/B on config3 (the current build, twice), digest
# compared with the reference run's 8b6bebe923b7187a.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-ab1}
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  AB_OPT=0 AB_CASES=16384:1 AB_REPS=3 timeout -k 10 200 python -u tools/ab_w.py > $O/ab_$i.log 2>&1 \
    || { echo "ab failed"; tail -20 $O/ab_$i.log; exit 1; }
  echo "run $i: $(grep 'W=16384' $O/ab_$i.log)"
done
