#!/bin/bash
# Round 3 hot-kernel A/B: (library, tuning) combinations on the full config3
# launch (tools/ab_w.py: best of AB_REPS, output digest -- must agree).
#   AB_RUNS="cur: cur:3=1 addtid: addtid:3=1"   lib name ('cur' = the in-tree
#   build, else ab/libdpathsim_<name>.so) and AB_TUNE after the colon.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03ab}
mkdir -p $O
export AB_CASES=${AB_CASES:-16384:1} AB_REPS=${AB_REPS:-3}
for run in ${AB_RUNS:-cur:}; do
  lib=${run%%:*}; tune=${run#*:}
  if [ "$lib" = cur ]; then L=$PWD/distributed-pathsim_amd/dpathsim/libdpathsim.so; else L=$PWD/ab/libdpathsim_$lib.so; fi
  n="${lib}_${tune//[=,]/-}"
  DPATHSIM_LIB=$L AB_TUNE=$tune timeout -k 10 300 python -u tools/ab_w.py > $O/ab_$n.log 2>&1 \
    || { echo "ab $n failed"; tail -30 $O/ab_$n.log; exit 1; }
  echo "$n:"; grep -v amdgpu.ids $O/ab_$n.log
done
# heavy-venue table sizes (venue skipping) with the in-tree library
for nh in ${AB_NHEAVY_LIST:-}; do
  AB_NHEAVY=$nh timeout -k 10 300 python -u tools/ab_w.py > $O/ab_nheavy$nh.log 2>&1 || { echo "ab nheavy $nh failed"; tail -30 $O/ab_nheavy$nh.log; exit 1; }
  echo "n_heavy $nh:"; grep -v amdgpu.ids $O/ab_nheavy$nh.log
done
