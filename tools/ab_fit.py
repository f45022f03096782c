"""Bitwise check + timing of whole fits across library builds (development tool).
usage: AB_LIBS=a.so,b.so[@VAR=val] python tools/ab_fit.py
Each library runs in its own process on the same seeded designs (CASES below: K1r at p = 256,
K1 at p = 128, the narrow kernel at p = 48, binomial fitSingle / fitMultiple, Poisson); for each
case it hashes the fit (iterations, coefficients, standard errors, deviance, null deviance,
Pearson, loglik) and reports the first pass's kernel time (the initial pass) and the fit's wall
time.  Prints whether every library's fits are bitwise the first one's."""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = os.environ.get("AB_CASES", "0:4000000:256:binomial:logit:multiple,0:4000000:256:binomial:logit:single,"
                       "0:6000000:128:binomial:probit:multiple,0:20000000:48:binomial:logit:multiple,"
                       "2:4000000:256:poisson:log:multiple")
code = r'''
import sys, os, time, hashlib, numpy as np
sys.path.insert(0, %r)
from sparkglm_amd import Engine
for case in os.environ["AB_CASES"].split(","):
    kind, n, p, fam, lnk, init = case.split(":")
    e = Engine(0)
    e.synth(int(kind), 0, int(n), int(p), 7)
    e.fit_glm(fam, lnk, init=init)  # warm
    e.reset_stats()
    t0 = time.perf_counter()
    f = e.fit_glm(fam, lnk, init=init)
    wall = time.perf_counter() - t0
    st = e.stats()
    h = hashlib.sha1()
    for v in (f.coefs, f.stderr, [f.deviance, f.null_deviance, f.pearson, f.loglik, float(f.iter)]):
        h.update(np.ascontiguousarray(np.asarray(v, dtype=np.float64)).tobytes())
    print("CASE", case, h.hexdigest()[:16], "%%.3f" %% (st["pass_kernel_ms"] / max(st["passes"], 1)), "%%.4f" %% wall, f.iter, flush=True)
    e.close()
''' % ROOT
libs = [l for l in os.environ.get("AB_LIBS", "").split(",") if l]
res, hashes = {}, {}
for rep in range(int(os.environ.get("AB_REPS", "2"))):
    for l in libs:
        lib, _, kv = l.partition("@")
        env = dict(os.environ, SGLM_LIB=os.path.join(ROOT, lib), AB_CASES=CASES)
        if kv:
            env[kv.split("=")[0]] = kv.split("=")[1]
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
        if out.returncode:
            print(l, "FAILED", out.stderr[-1500:], flush=True)
            sys.exit(1)
        for line in out.stdout.splitlines():
            if not line.startswith("CASE"):
                continue
            _, case, h, ms, wall, it = line.split()
            hashes.setdefault((l, case), h)
            res.setdefault((l, case), []).append((float(ms), float(wall), int(it)))
for case in CASES.split(","):
    ref = hashes[(libs[0], case)]
    for l in libs:
        v = res[(l, case)]
        print(f"{case:40s} {l:45s} {'bitwise' if hashes[(l, case)] == ref else 'DIFFERENT'} iter {v[0][2]} "
              f"mean pass ms {min(x[0] for x in v):.3f}  fit s {' '.join('%.4f' % x[1] for x in v)}", flush=True)
