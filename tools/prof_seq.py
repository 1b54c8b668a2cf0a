"""Kernel durations in launch order from a rocprofv3 kernel-trace database
(run_results.db), from the N-th occurrence of the first kernel on, optionally
only those whose name matches a substring.
  python tools/prof_seq.py gpurun_out/p4/run_results.db [occurrence] [filter]"""
import re
import sqlite3
import sys

db = sys.argv[1]
occ = int(sys.argv[2]) if len(sys.argv) > 2 else 1
flt = sys.argv[3] if len(sys.argv) > 3 else ""
c = sqlite3.connect(db)
rows = c.execute("select name, start, end, grid_x from kernels order by start").fetchall()
names = [re.sub(r"\(anonymous namespace\)::", "", r[0]) for r in rows]
starts = [i for i, n in enumerate(names) if n == names[0]]
i0 = starts[min(occ, len(starts) - 1)]
tot = 0.0
for i in range(i0, len(rows)):
    n = re.sub(r"\(.*", "", names[i]).replace("void ", "")[:64]
    if flt and flt not in n:
        continue
    d = (rows[i][2] - rows[i][1]) / 1e3
    tot += d
    print(f"{d:9.1f} {rows[i][3]:>10} {n}")
print(f"{tot:9.1f} us total")
