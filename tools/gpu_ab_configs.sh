set -u
bash tools/gpu_ab_w.sh && \
AB_CONFIG=config4 AB_CASES=32768:4,8192:1,4096:1 AB_REPS=1 timeout -k 10 300 python -u tools/ab_w.py > gpurun_out/ab_w4.log 2>&1 && cat gpurun_out/ab_w4.log && \
AB_CONFIG=config5 AB_CASES=32768:4,8192:1 AB_REPS=1 timeout -k 10 400 python -u tools/ab_w.py > gpurun_out/ab_w5.log 2>&1 && cat gpurun_out/ab_w5.log
