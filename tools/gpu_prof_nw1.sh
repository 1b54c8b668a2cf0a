#!/bin/bash
# Phase breakdown (shader clocks) + ablations/counters of the hot kernel at W=8192 (profiling build).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export DPATHSIM_LIB=$PWD/distributed-pathsim_amd/dpathsim/libdpathsim_prof.so
AB_W=8192 timeout -k 10 200 python3 -u tools/prof_phases.py > gpurun_out/phases_nw1.log 2>&1 || { echo "phases failed"; tail -20 gpurun_out/phases_nw1.log; exit 1; }
cat gpurun_out/phases_nw1.log
AB_W=8192 AB_ABLATE=1,2,4 timeout -k 10 200 python3 -u tools/ab_hot.py > gpurun_out/cnt_nw1.log 2>&1 || { echo "counters failed"; tail -20 gpurun_out/cnt_nw1.log; exit 1; }
cat gpurun_out/cnt_nw1.log
