"""Wide-path timing probe: for each (n, p) synth a logit design, run K IRLS iterations and
print the per-pass row-kernel / Gram-kernel / reduce / solve times and the Gram TFLOP/s."""
import os, sys, json, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparkglm_amd import Engine
k = int(os.environ.get("PK", "3"))
cases = [tuple(int(v) for v in c.split("x")) for c in os.environ.get("PCASES", "4000000x512,1000000x2048").split(",")]
e = Engine(0)
for n, p in cases:
    e.synth(0, 0, n, p, 5)
    beta = np.zeros(p)
    beta, _ = e.irls_iterations(beta, 1)
    e.reset_stats()
    t0 = time.perf_counter()
    beta, _ = e.irls_iterations(beta, k)
    dt = time.perf_counter() - t0
    s = e.stats()
    P = s["passes"]
    g = s["gram_kernel_ms"] / P
    r = s["row_kernel_ms"] / P
    flops = n * (p * (p + 1) + 2 * p)
    print(json.dumps({"n": n, "p": p, "path": s["path"], "items": s["workgroups"], "gram_ms": g, "row_ms": r,
                      "reduce_ms": s["reduce_kernel_ms"] / P, "solve_ms": s["solve_ms"] / k,
                      "step_ms": dt * 1e3 / k, "gram_tflops": flops / g / 1e9,
                      "row_gbs": n * 8 * (p + 3) / r / 1e6 if r > 0 else None,
                      "pass_tflops": flops / (g + r) / 1e9}), flush=True)
