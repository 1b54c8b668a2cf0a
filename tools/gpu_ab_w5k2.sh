#!/bin/bash
# config5 (top-100, two top-k registers per lane): 4 waves per SIMD (current)
# vs 5 waves per SIMD with the register budget forced to 96 (ab/libdpathsim_w5k2.so,
# built first with: tools/build_lean_variant.sh w5k2 -DDPS_W5_KPL=2).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export AB_CONFIG=config5 AB_CASES=8192:1 AB_REPS=2
timeout -k 10 400 python -u tools/ab_w.py > gpurun_out/ab_k2_cur.log 2>&1 || { echo "cur failed"; tail -20 gpurun_out/ab_k2_cur.log; exit 1; }
grep " ms " gpurun_out/ab_k2_cur.log
DPATHSIM_LIB=$PWD/ab/libdpathsim_w5k2.so timeout -k 10 400 python -u tools/ab_w.py > gpurun_out/ab_k2_w5.log 2>&1 || { echo "w5 failed"; tail -20 gpurun_out/ab_k2_w5.log; exit 1; }
grep " ms " gpurun_out/ab_k2_w5.log
