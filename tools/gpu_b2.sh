set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 900 --timeout-method thread > gpurun_out/pytest_gpu_b2.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu_b2.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_b2.log
AB_ENV="DPATHSIM_TILE_LPB=1024;DPATHSIM_TILE_LPB=2048;DPATHSIM_TILE_LPB=4096;DPATHSIM_TILE_LPB=8192" timeout -k 10 300 python -u tools/build_ab.py > gpurun_out/build_ab.log 2>&1 || { echo "build_ab failed"; tail -20 gpurun_out/build_ab.log; exit 1; }
cat gpurun_out/build_ab.log | grep env
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_b2.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_b2.log; exit 1; }
tail -1 gpurun_out/bench_b2.log
