"""A/B timing of in-tree library builds on the same GPU (development tool).
usage: AB_LIBS=sparkglm_amd/lib_ab/base.so,sparkglm_amd/lib/libsglm_hip.so[@VAR=val...] AN=.. AP=.. AK=.. AF=.. AL=.. python tools/ab.py
Runs each library twice, alternating, and prints the mean pass time of 3 passes per run."""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import sys, os, numpy as np
sys.path.insert(0, %r)
from sparkglm_amd import Engine
n, p, k = int(os.environ.get("AN", "20000000")), int(os.environ.get("AP", "256")), int(os.environ.get("AK", "0"))
fam, lnk = os.environ.get("AF", "binomial"), os.environ.get("AL", "logit")
e = Engine(0); e.synth(k, 0, n, p, 2)
b = np.full(p, 0.01)
if k == 3: b[0] = 1.0
e.irls_pass(b, family=fam, link=lnk); e.reset_stats()
for _ in range(4): e.irls_pass(b, family=fam, link=lnk)
s = e.stats(); P = s["passes"]
ms = s["pass_kernel_ms"] / P  # fused / narrow: the pass kernel; wide: row + Gram kernels
print("%%.3f" %% ms)
''' % ROOT
libs = [l for l in os.environ.get("AB_LIBS", "").split(",") if l] or [os.path.join(ROOT, "sparkglm_amd/lib/libsglm_hip.so")]
n, p = int(os.environ.get("AN", "20000000")), int(os.environ.get("AP", "256"))
res = {l: [] for l in libs}
for rep in range(int(os.environ.get("AB_REPS", "2"))):
    for l in libs:
        # "path@VAR=val@VAR2=val2": that library with extra environment (e.g. @SGLM_FUSED_SPLIT=6)
        path, *kv = l.split("@")
        env = dict(os.environ, SGLM_LIB=os.path.join(ROOT, path), **dict(x.split("=", 1) for x in kv))
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
        if out.returncode:
            print(l, "FAILED", out.stderr[-500:], flush=True)
            sys.exit(1)
        res[l].append(float(out.stdout.strip().split()[-1]))
for l, v in res.items():
    ms = min(v)
    print(f"{os.path.basename(os.path.dirname(l.split('@')[0])) + '/' + os.path.basename(l):48s} n={n} p={p}: pass ms {' '.join('%.3f' % x for x in v)}  "
          f"best {ms:.3f}  {n * p * (p + 3) / ms / 1e9:.1f} TF", flush=True)
