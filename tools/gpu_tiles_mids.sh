#!/bin/bash
# Many-mid tile build: GPU tests of the mid-range block path, then the build
# phases of config4 / config5 with the block path and the global-atomic path.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_synth.py tests/test_gpu_edge.py tests/test_gpu_fullsize.py -m gpu -x -v \
  --timeout 500 --timeout-method thread -k "many_mids or config4 or config5 or spgemm_long" > gpurun_out/pytest_tiles_mids.log 2>&1 \
  || { echo "pytest failed"; tail -40 gpurun_out/pytest_tiles_mids.log; exit 1; }
tail -3 gpurun_out/pytest_tiles_mids.log
for c in config4 config5; do
  AB_CONFIG=$c AB_REPS=5 AB_ENV="DPATHSIM_TILE_GLOBAL=1;DPATHSIM_TILE_GLOBAL=0" timeout -k 10 300 python -u tools/build_ab.py \
    > gpurun_out/build_ab_tiles_$c.log 2>&1 || { echo "build_ab $c failed"; tail -20 gpurun_out/build_ab_tiles_$c.log; exit 1; }
  grep phase gpurun_out/build_ab_tiles_$c.log
done
