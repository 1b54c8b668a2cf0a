#!/bin/bash
# The in-tree library with the optimistic passes off (the engine default) and
# on, beside every ab/libdpathsim_*.so; ABAB order, config3 full eng.topk.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-ab4x}
mkdir -p $O
export AB_CASES=${AB_CASES:-16384:1} AB_REPS=${AB_REPS:-3}
for round in 1 2; do
  for o in 0 1; do
    AB_OPT=$o timeout -k 10 300 python -u tools/ab_w.py > $O/ab_tree_opt${o}_$round.log 2>&1 \
      || { echo "ab tree failed"; tail -30 $O/ab_tree_opt${o}_$round.log; exit 1; }
    echo "tree opt=$o #$round: $(grep 'digest' $O/ab_tree_opt${o}_$round.log)"
  done
  for lib in ab/libdpathsim_*.so; do
    n=$(basename $lib .so); n=${n#libdpathsim_}
    DPATHSIM_LIB=$PWD/$lib timeout -k 10 300 python -u tools/ab_w.py > $O/ab_${n}_$round.log 2>&1 \
      || { echo "ab $n failed"; tail -30 $O/ab_${n}_$round.log; exit 1; }
    echo "$n #$round: $(grep 'digest' $O/ab_${n}_$round.log)"
  done
done
