"""Static instruction counts of one kernel in a `hipcc -g -S` listing, by the
source line (.loc) each instruction belongs to and by class -- a map of where
the hot kernel's code goes (round 5; no PC sampling on this pool).
usage: isa_lines.py listing.s kernel_symbol [top]"""
import collections, re, sys

path, sym = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 60
files, cur = {}, None
rows = collections.defaultdict(collections.Counter)
inside = False
for ln in open(path):
    m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', ln)
    if m:
        files[m.group(1)] = m.group(2)
        continue
    if ln.startswith(sym + ":"):
        inside = True
        continue
    if not inside:
        continue
    m = re.match(r'\s*\.loc\s+(\d+)\s+(\d+)', ln)
    if m:
        cur = f"{files.get(m.group(1), m.group(1))}:{m.group(2)}"
        continue
    m = re.match(r'\s+([a-z][a-z0-9_]+)', ln)
    if not m or ln.lstrip().startswith((".", ";")):
        continue
    op = m.group(1)
    cls = ("spill" if op in ("v_writelane_b32",) else
           "readlane" if op == "v_readlane_b32" else
           "VALU" if op.startswith("v_") else
           "nop" if op == "s_nop" else
           "branch" if op.startswith("s_cbranch") or op == "s_branch" else
           "waitcnt" if op.startswith("s_waitcnt") else
           "SMEM" if op.startswith(("s_load", "s_buffer")) else
           "SALU" if op.startswith("s_") else
           "LDS" if op.startswith("ds_") else
           "VMEM" if op.startswith(("global_", "buffer_", "flat_")) else "other")
    rows[cur][cls] += 1
    if op == "s_endpgm":
        break
tot = collections.Counter()
for c in rows.values():
    tot.update(c)
print("total", dict(tot))
keys = ["VALU", "readlane", "spill", "SALU", "branch", "nop", "waitcnt", "LDS", "VMEM", "SMEM"]
print(f"{'line':34s}" + "".join(f"{k:>9s}" for k in keys))
for line, c in sorted(rows.items(), key=lambda kv: -sum(kv[1].values()))[:top]:
    print(f"{str(line):34s}" + "".join(f"{c[k]:9d}" for k in keys))
