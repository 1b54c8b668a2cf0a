#!/bin/bash
# Round 5: hot-kernel A/B on config5 (k = 100, the KPL = 2 instantiation) for
# the libraries named in AB_LIBS (default: base w5), twice each.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-ab5c5}
mkdir -p $O
export AB_CONFIG=config5 AB_CASES=${AB_CASES:-16384:1} AB_REPS=${AB_REPS:-2} AB_OPT=0
for round in 1 2; do
  for n in ${AB_LIBS:-base w5}; do
    DPATHSIM_LIB=$PWD/ab/libdpathsim_$n.so timeout -k 10 400 python -u tools/ab_w.py > $O/ab_${n}_$round.log 2>&1 \
      || { echo "ab $n failed"; tail -30 $O/ab_${n}_$round.log; exit 1; }
    echo "$n #$round: $(grep 'digest' $O/ab_${n}_$round.log | cut -c1-140)"
  done
done
