"""Bitwise check + A/B timing of fused-pass (p = 256) builds (development tool).
usage: AB_LIBS=a.so,b.so[@VAR=val] AN=.. AP=.. python tools/ab_k1r.py
(lib@VAR=val runs that library with the environment variable set, e.g. lib.so@SGLM_FUSED_SPLIT=0)
Each library runs in its own process on the same seeded design: one IRLS pass at a fixed beta
(the packed X'WX | X'Wz | scalars saved), then the mean pass time over 4 passes.  Prints whether
every library's pass output is bitwise the first one's, and the timings, alternating REPS times."""
import os, subprocess, sys, hashlib
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import sys, os, numpy as np, hashlib
sys.path.insert(0, %r)
from sparkglm_amd import Engine
n, p, k = int(os.environ.get("AN", "2000000")), int(os.environ.get("AP", "256")), int(os.environ.get("AK", "0"))
fam, lnk = os.environ.get("AF", "binomial"), os.environ.get("AL", "logit")
e = Engine(0); e.synth(k, 0, n, p, 2)
b = np.linspace(-0.02, 0.02, p)
if k == 3: b[0] = 1.0
g, xz, s = e.irls_pass(b, family=fam, link=lnk)
h = hashlib.sha1(np.ascontiguousarray(g).tobytes() + np.ascontiguousarray(xz).tobytes() + np.float64(s).tobytes()).hexdigest()[:16]
if os.environ.get("AB_SAVE"):
    np.save(os.environ["AB_SAVE"], np.concatenate([np.ravel(g), np.ravel(xz), np.ravel(np.float64(s))]))
e.reset_stats()
for _ in range(4): e.irls_pass(b, family=fam, link=lnk)
st = e.stats()
print(h, "%%.3f" %% (st["pass_kernel_ms"] / st["passes"]))
''' % ROOT
libs = [l for l in os.environ.get("AB_LIBS", "").split(",") if l] or [os.path.join(ROOT, "sparkglm_amd/lib/libsglm_hip.so")]
n, p = int(os.environ.get("AN", "2000000")), int(os.environ.get("AP", "256"))
res = {l: [] for l in libs}
hashes = {}
allh = {}
for rep in range(int(os.environ.get("AB_REPS", "2"))):
    for l in libs:
        lib, _, kv = l.partition("@")
        env = dict(os.environ, SGLM_LIB=os.path.join(ROOT, lib), AB_SAVE=f"/tmp/ab_out_{libs.index(l)}.npy")
        if kv:
            env[kv.split("=")[0]] = kv.split("=")[1]
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
        if out.returncode:
            print(l, "FAILED", out.stderr[-800:], flush=True)
            sys.exit(1)
        h, ms = out.stdout.strip().split()[-2:]
        hashes.setdefault(l, h)
        allh.setdefault(l, set()).add(h)
        res[l].append(float(ms))
ref = hashes[libs[0]]
import numpy as np
o0 = np.load("/tmp/ab_out_0.npy")
def relmax(i):
    o = np.load(f"/tmp/ab_out_{i}.npy")
    d = np.abs(o - o0) / np.maximum(np.abs(o0), 1e-300)
    return float(np.nanmax(d)) if d.size else 0.0
for l, v in res.items():
    ms = min(v)
    print(f"{l:50s} n={n} p={p}: {'bitwise' if hashes[l] == ref else 'DIFFERENT %s (max rel %.1e)' % (hashes[l], relmax(libs.index(l)))} pass ms "
          f"{' '.join('%.3f' % x for x in v)}  best {ms:.3f}  {n * p * (p + 3) / ms / 1e9:.1f} TF"
          f"{'  (run-to-run: %d distinct hashes)' % len(allh[l]) if len(allh[l]) > 1 else ''}", flush=True)
