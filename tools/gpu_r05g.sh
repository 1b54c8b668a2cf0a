#!/bin/bash
# Round 5: build-side A/B (every abb/libdpathsim_*.so: device build phases on
# config3 at W = 16384 and config4 at W = 8192, tools/build_ab.py), after the
# GPU tests of the build kernels with the in-tree library.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05g}
mkdir -p $O
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_spgemm_mids.py tests/test_gpu_edge.py tests/test_gpu_synth.py \
    -x -q --timeout 300 --timeout-method thread > $O/pytest_build.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest_build.log; exit 1; }
  tail -2 $O/pytest_build.log
fi
for cfg in config3:16384 config4:8192; do
  for lib in abb/libdpathsim_*.so; do
    n=$(basename $lib .so); n=${n#libdpathsim_}
    DPATHSIM_LIB=$PWD/$lib AB_CONFIG=${cfg%:*} AB_W=${cfg#*:} AB_REPS=${AB_REPS:-7} timeout -k 10 300 \
      python -u tools/build_ab.py > $O/build_${cfg%:*}_$n.log 2>&1 || { echo "build_ab $n failed"; tail -20 $O/build_${cfg%:*}_$n.log; exit 1; }
    echo "${cfg%:*} $n: $(grep phase_ms $O/build_${cfg%:*}_$n.log | cut -c1-400)"
  done
done
