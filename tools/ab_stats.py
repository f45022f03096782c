"""Same-box A/B of the narrow pass's final statistics: the default (Poisson / Gamma: in the
deviance-only last pass), in every pass (SGLM_STATS_EVERY_PASS=1), the eta store + stats_kernel
(SGLM_ETA_STORE=1): per-iteration pass-kernel ms (irls_iterations, as the
bench times them) and time to converge, alternating, on one synthetic shard per engine.
  python tools/ab_stats.py [kind rows p family link reps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparkglm_amd import Engine  # noqa: E402

kind, n, p = int(sys.argv[1]) if len(sys.argv) > 1 else 2, int(float(sys.argv[2])) if len(sys.argv) > 2 else 125_000_000, \
    int(sys.argv[3]) if len(sys.argv) > 3 else 64
fam = sys.argv[4] if len(sys.argv) > 4 else "poisson"
lnk = sys.argv[5] if len(sys.argv) > 5 else "log"
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 3
engs = {}
for label, env, every in (("default", "0", "0"), ("stats_every_pass", "0", "1"), ("eta_store", "1", "0")):
    os.environ["SGLM_ETA_STORE"] = env
    os.environ["SGLM_STATS_EVERY_PASS"] = every
    e = Engine(0)
    e.synth(kind, 0, n, p, 3)
    engs[label] = e
res = {k: {"pass_ms": [], "ttc_s": []} for k in engs}
fits = {}
for r in range(reps):
    for label, e in engs.items():
        t0 = time.perf_counter()
        f = e.fit_glm(fam, lnk)
        ttc = time.perf_counter() - t0
        fits[label] = f
        e.reset_stats()
        e.irls_iterations(np.array(f.coefs), 5, fam, lnk)
        st = e.stats()
        res[label]["pass_ms"].append(st["pass_kernel_ms"] / st["passes"])
        res[label]["ttc_s"].append(ttc)
a, b = fits["default"], fits["eta_store"]
print(f"{fam}/{lnk} {n} x {p}")
for k, v in res.items():
    print(f"  {k:14s} pass ms {np.round(v['pass_ms'], 3).tolist()}  ttc s {np.round(v['ttc_s'], 4).tolist()}")
rel = lambda x, y: float(np.max(np.abs(np.asarray(x) - np.asarray(y)) / np.abs(np.asarray(y))))
print(f"  same fit: iter {a.iter}/{b.iter} coefs {rel(a.coefs, b.coefs):.1e} dev {rel(a.deviance, b.deviance):.1e} "
      f"pearson {rel(a.pearson, b.pearson):.1e} loglik {rel(a.loglik, b.loglik):.1e}")
