"""Small fused-pass workload for rocprofv3 (kernel trace / PMC): PN x PP design of synth kind
PKIND fitted as PF/PL, PK passes (PLM=1: PK LM fits instead)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparkglm_amd import Engine
n, p, k = int(os.environ.get("PN", "20000000")), int(os.environ.get("PP", "256")), int(os.environ.get("PK", "3"))
kind = int(os.environ.get("PKIND", "0"))
fam, lnk = os.environ.get("PF", "binomial"), os.environ.get("PL", "logit")
e = Engine(0)
e.synth(kind, 0, n, p, 2, procedural=os.environ.get("PPROC", "0") == "1")
b = np.full(p, 0.01)
for _ in range(k):
    if os.environ.get("PLM", "0") == "1":  # LM.fit (the one-pass LM Gram of the device round trip)
        e.fit_lm()
    else:
        e.irls_pass(b, family=fam, link=lnk)
s = e.stats()
print("pass ms", s["pass_kernel_ms"] / s["passes"], "n", n, "p", p, "path", s["path"])
