#!/bin/bash
# Rehearse bench.py's multi-rank path on a one-GPU box: 2 ranks on cuda:0 over gloo
# (the driver's N>1 runs use one GPU per rank and RCCL).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
DPATHSIM_BENCH_DEVICE=0 DPATHSIM_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run \
  --nnodes=1 --nproc-per-node ${NR:-2} --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus ${NR:-2} --steps 2 --warmup 1 \
  > gpurun_out/bench_rehearse${NR:-2}.log 2>&1 || { echo "rehearsal failed"; tail -30 gpurun_out/bench_rehearse${NR:-2}.log; exit 1; }
grep '"metric"' gpurun_out/bench_rehearse${NR:-2}.log
