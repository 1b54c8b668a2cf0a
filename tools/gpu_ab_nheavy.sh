#!/bin/bash
# Venue skipping: heavy venues in the dense table (engine.n_heavy) swept on the
# full config3 launch, then every ab/libdpathsim_*.so variant; time + digest.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-abnh}
mkdir -p $O
export AB_CASES=16384:1 AB_REPS=2 AB_OPT=0
for nh in ${NHS:-16 32 48 64}; do
  AB_NHEAVY=$nh timeout -k 10 300 python -u tools/ab_w.py > $O/nh_$nh.log 2>&1 || { echo "nh $nh failed"; tail -20 $O/nh_$nh.log; exit 1; }
  echo "n_heavy $nh: $(grep digest $O/nh_$nh.log)"
done
for round in 1 2; do
  for lib in ab/libdpathsim_*.so; do
    n=$(basename $lib .so); n=${n#libdpathsim_}
    DPATHSIM_LIB=$PWD/$lib timeout -k 10 300 python -u tools/ab_w.py > $O/ab_${n}_$round.log 2>&1 \
      || { echo "ab $n failed"; tail -30 $O/ab_${n}_$round.log; exit 1; }
    echo "$n #$round: $(grep 'digest' $O/ab_${n}_$round.log)"
  done
done
