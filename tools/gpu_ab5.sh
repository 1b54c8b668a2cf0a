#!/bin/bash
# Round-5 hot-kernel A/B: every ab/libdpathsim_*.so in turn, twice (ABAB order
# against drift), full config3 eng.topk at the engine default (W = 16384,
# optimistic passes off), time + output digest per library (tools/ab_w.py).
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-ab5}
mkdir -p $O
export AB_CASES=${AB_CASES:-16384:1} AB_REPS=${AB_REPS:-3} AB_OPT=${AB_OPT:-0}
for round in 1 2; do
  for lib in ab/libdpathsim_*.so; do
    n=$(basename $lib .so); n=${n#libdpathsim_}
    DPATHSIM_LIB=$PWD/$lib timeout -k 10 300 python -u tools/ab_w.py > $O/ab_${n}_$round.log 2>&1 \
      || { echo "ab $n failed"; tail -30 $O/ab_${n}_$round.log; exit 1; }
    echo "$n #$round: $(grep 'digest' $O/ab_${n}_$round.log | cut -c1-140)"
  done
done
