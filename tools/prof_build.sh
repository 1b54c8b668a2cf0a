#!/bin/bash
# rocprofv3 kernel trace of the device build (tools/build_ab.py, one setting):
# per-kernel average durations -> gpurun_out/prof_build_summary.txt
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_build
AB_REPS=3 AB_ENV="${AB_ENV:-X=1}" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d gpurun_out/prof_build -o run -- python3 -u tools/build_ab.py > gpurun_out/prof_build.log 2>&1 \
  || { echo "prof failed"; tail -20 gpurun_out/prof_build.log; exit 1; }
python3 - <<'PY' | tee gpurun_out/prof_build_summary.txt
import csv, glob, re
f = glob.glob("gpurun_out/prof_build/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    m = re.search(r"(k_[a-z0-9_]+(<[^>]*>)?|[A-Za-z_]*kernel[A-Za-z_0-9]*|__amd[a-zA-Z_]+)", n)
    print(f"{(m.group(1) if m else n[:50]):50s} calls {int(r['Calls']):5d} avg {float(r['AverageNs'])/1e3:9.1f} us  total {float(r['TotalDurationNs'])/1e6:8.2f} ms")
PY
