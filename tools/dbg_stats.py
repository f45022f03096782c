import os, sys
sys.path.insert(0, '/root/repo')
import numpy as np
from sparkglm_amd import Engine
for env in ("0", "1"):
    os.environ["SGLM_ETA_STORE"] = env
    e = Engine(0)
    e.synth(2, 0, 2_000_000, 64, 3)
    f = e.fit_glm("poisson", "log")
    g, xz, s = e.irls_pass(f.coefs, family="poisson", link="log")
    print("ETA_STORE", env, "pearson", repr(f.pearson), "ll", repr(f.loglik), "pass scalars", s.tolist())
    e.close()
