"""GPU side of oracle/gram_split.py: the engine's X'WX / X'Wz on the full configs[3] shard
(12.5M x 2048 gamma / inverse) at the oracle's final coefficients, the engine's own Cholesky solve
of it, and the engine's fit -- written to gpurun_out/gram_split/engine.npz for the CPU comparison.

    python tools/gram_split_capture.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from sparkglm_amd import Engine  # noqa: E402


def main():
    c = json.load(open(os.path.join(ROOT, "tests", "golden", "full_scale.json")))["gamma2048"]
    beta = np.asarray(c["coefs"])
    out = os.path.join(ROOT, "gpurun_out", "gram_split")
    os.makedirs(out, exist_ok=True)
    t0 = time.time()
    with Engine(0) as e:
        e.synth(c["kind"], c["row0"], c["n"], c["p"], c["seed"])
        print(f"shard generated {time.time() - t0:.1f} s", flush=True)
        f = e.fit_glm(c["family"], c["link"], tol=c["tol"])
        print(f"fit: {f.iter} iterations, deviance {f.deviance!r}", flush=True)
        G, xtwz, s = e.irls_pass(beta, family=c["family"], link=c["link"])
        x_chol, dev = e.irls_iterations(beta, 1, c["family"], c["link"])  # pass at beta + the device solve
        st = e.stats()
    # the engine's LU route (SGLM_WIDE_SOLVE=lu: rocSOLVER getrf + getri, coefs = inv * X'Wz in order)
    os.environ["SGLM_WIDE_SOLVE"] = "lu"
    with Engine(0) as e:
        e.synth(c["kind"], c["row0"], c["n"], c["p"], c["seed"])
        x_lu_roc, _ = e.irls_iterations(beta, 1, c["family"], c["link"])
        assert e.stats()["solve_path_name"] == "device-lu"
    del os.environ["SGLM_WIDE_SOLVE"]
    p = G.shape[0]
    i, j = np.tril_indices(p)
    packed = np.empty(p * (p + 1) // 2)
    packed[i * (i + 1) // 2 + j] = G[i, j]
    np.savez(os.path.join(out, "engine.npz"), beta=beta, G=packed, xtwz=xtwz, s=s, x_chol=x_chol, x_lu_roc=x_lu_roc,
             fit_coefs=f.coefs, fit_iter=f.iter, solve_path=st["solve_path_name"])
    print(f"solve path {st['solve_path_name']}; saved in {time.time() - t0:.1f} s", flush=True)


if __name__ == "__main__":
    main()
