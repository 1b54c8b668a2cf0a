#!/bin/bash
# Round 4: dist entry points (dps_shard_edges / dps_pack_counts /
# dps_unpack_gathered) on the box -- GPU tests of test_dist, a 2-rank gloo
# rehearsal of bench.py's N > 1 step, then N = 1 bench.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-r04b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_dist.py tests/test_gpu_logvectors.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $O/pytest_dist.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_dist.log; exit 1; }
tail -2 $O/pytest_dist.log
DPATHSIM_BENCH_DEVICE=0 DPATHSIM_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 \
  --no-cpu-baseline > $O/bench_rehearse2.log 2>&1 || { echo "rehearsal failed"; tail -30 $O/bench_rehearse2.log; exit 1; }
grep '"metric"' $O/bench_rehearse2.log | cut -c1-300
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench1.log 2>&1 \
  || { echo "bench failed"; tail -30 $O/bench1.log; exit 1; }
grep '"metric"' $O/bench1.log | cut -c1-400
