"""Profiling tool: time the fused pass with parts ablated (SGLM_DEBUG_ABLATE bits:
1 row stage, 2 MFMA, 4 DMA, 8 eta dot product, 16 trivial family arithmetic, 32 no eta store),
on the ablation build (make -C sparkglm_amd/csrc ablate).
AN rows, AP columns, AK synth kind, AF/AL family/link."""
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
e.irls_pass(b, family=fam, link=lnk); e.reset_stats()
for _ in range(3): e.irls_pass(b, family=fam, link=lnk)
s = e.stats(); P = s["passes"]
nv = 3 if k == 2 else 1
ms = s["pass_kernel_ms"] / P
print("pass %%.3f ms  %%.0f GB/s  %%.1f TF  wg %%d" %% (ms, n * (8 * p + 8 * nv) / ms / 1e6, n * p * (p + 3) / ms / 1e9, s["workgroups"]))
''' % ROOT
for bits in [int(b) for b in os.environ.get("ABITS", "0,1,2,4,3,8,16").split(",")]:
    env = dict(os.environ, SGLM_DEBUG_ABLATE=str(bits))
    env.setdefault("SGLM_LIB", os.path.join(ROOT, "sparkglm_amd", "lib_ablate", "libsglm_hip.so"))  # make ablate
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    print(f"ablate={bits:3d}: {out.stdout.strip()} {out.stderr[-300:] if out.returncode else ''}", flush=True)
