#!/bin/bash
# Round 5: kernel variant A/B, then the GPU tests that exercise the hot
# kernel's rarer paths (wide passes, > 64 venues, venue skipping, splits).
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-r05f}
mkdir -p $O
export TMPDIR=/tmp
TAG=${TAG:-r05f}_ab bash tools/gpu_ab5.sh || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py::test_crafted_wide_passes tests/test_gpu_venue_skip.py \
  tests/test_gpu_synth.py tests/test_gpu_edge.py tests/test_gpu_counters.py -m gpu -x -q \
  --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
