#!/bin/bash
# Round 5: hot-kernel variant A/B, then the split-build scaling prediction.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-r05e}
mkdir -p $O
export TMPDIR=/tmp
TAG=${TAG:-r05e}_ab bash tools/gpu_ab5.sh || exit 1
timeout -k 10 600 python -u tools/split_balance.py > $O/split_balance.txt 2>&1 \
  || { echo "split_balance failed"; tail -30 $O/split_balance.txt; exit 1; }
grep '"world"' $O/split_balance.txt | cut -c1-400
