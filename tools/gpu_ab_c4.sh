set -u
cd /root/repo
mkdir -p gpurun_out
AB_CONFIG=config4 AB_REPS=5 AB_ENV="DPATHSIM_SPGEMM=hash;DPATHSIM_SPGEMM=sort" timeout -k 10 300 python -u tools/build_ab.py > gpurun_out/build_ab_c4sort.log 2>&1 || { tail -20 gpurun_out/build_ab_c4sort.log; exit 1; }
grep phase gpurun_out/build_ab_c4sort.log
