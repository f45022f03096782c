"""Profiling tool: time the fused pass with parts ablated (SGLM_DEBUG_ABLATE bits)."""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import sys, os, numpy as np
sys.path.insert(0, %r)
from sparkglm_amd import Engine
n, p = int(os.environ.get("AN", "20000000")), int(os.environ.get("AP", "256"))
e = Engine(0); e.synth(0, 0, n, p, 2)
b = np.full(p, 0.01)
e.irls_pass(b); e.reset_stats()
for _ in range(3): e.irls_pass(b)
s = e.stats(); print("pass %%.3f gram %%.3f" %% (s["pass_kernel_ms"] / s["passes"], s["gram_kernel_ms"] / s["passes"]))
''' % ROOT
for bits in [int(b) for b in os.environ.get("ABITS", "0,1,2,4,3,5,6,7").split(",")]:
    env = dict(os.environ, SGLM_DEBUG_ABLATE=str(bits))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    print(f"ablate={bits} (1 row-stage, 2 mfma, 4 dma, 32 barriers, 64 lds operands): pass ms {out.stdout.strip()} {out.stderr[-300:] if out.returncode else ''}", flush=True)
