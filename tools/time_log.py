"""Throughput of the native all-pairs log writer on a config3-shaped result
(1M source rows x top-10, random targets/scores; host only)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-pathsim_amd"))
import numpy as np
from dpathsim.synth import synth_config
from dpathsim.logfmt import write_topk_log, AuthorStrings

cfg = sys.argv[1] if len(sys.argv) > 1 else "config3"
k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
threads = int(sys.argv[3]) if len(sys.argv) > 3 else 0
out = sys.argv[4] if len(sys.argv) > 4 else "/tmp/allpairs.log"
t = synth_config(cfg).typed()
na = t.n_authors
rng = np.random.default_rng(0)
idx = rng.integers(0, na, size=(na, k), dtype=np.int32)
cnt = rng.integers(1, 50, size=(na, k), dtype=np.int64)
g = rng.integers(1, 10 ** 7, size=na, dtype=np.int64)
score = 2 * cnt / (g[:, None] + g[idx])
t0 = time.perf_counter(); s = AuthorStrings(t); t1 = time.perf_counter()
write_topk_log(out, t, idx, cnt, score, g, append=False, stage_seconds=2.1e-11, overall_seconds=0.2,
               n_threads=threads, strings=s)
t2 = time.perf_counter()
sz = os.path.getsize(out)
print(f"{cfg}: {na} rows x top-{k}: strings {t1 - t0:.2f} s, write {t2 - t1:.2f} s, "
      f"{sz / 1e9:.2f} GB, {na * k * 5 / (t2 - t1) / 1e6:.1f} M lines/s, threads {threads or os.cpu_count()}")
os.remove(out)
