"""Kernels of the last of three builds in a rocprofv3 kernel trace
(tools/build_trace.py), in launch order, with durations (us).
usage: build_trace_summary.py run_kernel_trace.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
# a build starts with k_extract's predecessor fill; split on k_extract launches
starts = [i for i, r in enumerate(rows) if "k_extract(" in r["Kernel_Name"]]
first = starts[-1] - 1 if starts else 0
last = rows[first:]
tot = 0.0
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    name = r["Kernel_Name"].replace("dps::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} {d:8.1f}  {name[:70]}  grid {r.get('Grid_Size', r.get('Grid_Size_X', ''))}")
span = (int(last[-1]["End_Timestamp"]) - t0) / 1e3
print(f"kernels {len(last)}, busy {tot:.1f} us, span {span:.1f} us")
