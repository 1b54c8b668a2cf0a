"""Hot-kernel time by row class: the lightest fraction f of the author rows (by
sum_{v in x} n_v, the build's row_terms) against the rest, each as one
dps_cct_topk_rows launch, with the kernel's pass / chunk counts.  Tells how
much of the launch the light rows cost."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-pathsim_amd"))
import numpy as np
import torch

import dpathsim
from dpathsim.engine import PathSimEngine
from dpathsim.synth import CONFIGS, synth_config

cfg = os.environ.get("AB_CONFIG", "config3")
K = int(os.environ.get("AB_K", str(CONFIGS[cfg][4])))
fracs = [float(f) for f in os.environ.get("LS_FRACS", "0.1,0.2,0.33,0.5").split(",")]
t = synth_config(cfg).typed(dpathsim.METAPATHS[CONFIGS[cfg][3]])
NA = t.n_authors
eng = PathSimEngine(t)
eng.upload().build()
terms = eng.tensor("row_terms")[:NA].cpu().numpy()
order = np.argsort(terms, kind="stable")
q = np.quantile(terms, [0.1, 0.2, 0.33, 0.5, 0.9, 0.99])
print(f"{cfg}: NA={NA} sum terms {terms.sum():.4e} quantiles 10/20/33/50/90/99 % {q.tolist()}", flush=True)


def timed(rows):
    r = torch.from_numpy(rows.astype(np.int64)).cuda()
    eng.topk_rows(K, r[: min(len(rows), 2000)])
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(2):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        eng.topk_rows(K, r)
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best, eng.kernel_counts()


e0 = torch.cuda.Event(enable_timing=True)
e1 = torch.cuda.Event(enable_timing=True)
eng.topk(K)
e0.record()
eng.topk(K)
e1.record()
torch.cuda.synchronize()
kc = eng.kernel_counts()
print(f"all rows (eng.topk): {e0.elapsed_time(e1):.2f} ms passes {kc['passes']} chunks {kc['chunks']}",
      flush=True)
for f in fracs:
    n = int(f * NA)
    lo, hi = order[:n], order[n:]
    tl, kl = timed(lo)
    th, kh = timed(hi)
    print(f"f={f:.2f}: light {n} rows (terms <= {terms[order[n - 1]]}, sum {terms[lo].sum():.3e}) "
          f"{tl:.2f} ms passes {kl['passes']} chunks {kl['chunks']} | heavy {NA - n} rows "
          f"{th:.2f} ms passes {kh['passes']} chunks {kh['chunks']}", flush=True)
