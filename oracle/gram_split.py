"""configs[3] (gamma / inverse, p = 2048): where the engine's coefficient error comes from.

TEST INFRASTRUCTURE ONLY (the checker side; never imported by sparkglm_amd).

The engine's final coefficients on the full 12.5M x 2048 shard sit up to ~1e-7 (elementwise, on
the smallest coefficients) from the streaming oracle's, while norm-wise they agree at ~1e-12.  Two
things differ between the two fits' last solve (utils.scala:103-105, 134-136):
  (i)  the Gram X'WX / X'Wz itself -- summed in another order (fp64 MFMA tiles, fixed-order
       partial reduction) than the oracle's blocked loops;
  (ii) the solve -- the engine's rocSOLVER Cholesky (potrf / potrs) against Breeze inv's
       LU + explicit inverse (dgetrf + dgetri), which the oracle restates unblocked.
At ONE beta (the oracle's final coefficients, full_scale.json) this script separates them:
  a) G_engine vs G_oracle, entrywise and norm-wise                          -> (i) at the source
  b) x_chol(G_engine) [engine]  vs  x_lu(G_engine) [oracle's LU on the engine's Gram] -> (ii)
  c) x_lu(G_engine)  vs  x_lu(G_oracle)                                      -> (i) through the solve
so that x_chol(G_engine) - x_lu(G_oracle) = (ii) + (i).

    python oracle/gram_split.py oracle              # the streaming oracle's pass (~15 min, 8 cores)
                                                    #   -> oracle/build/gram_split_oracle.npz
    python oracle/gram_split.py compare ENGINE.npz  # ENGINE.npz from tools/gram_split_capture.py (GPU)
                                                    #   -> tests/golden/gram_split_p2048.{json,npz}
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
import pyoracle as po  # noqa: E402

CASE = "gamma2048"
NV = 8  # probe vectors of the committed digest G V


def full_scale_case():
    return json.load(open(os.path.join(ROOT, "tests", "golden", "full_scale.json")))[CASE]


def probe_vectors(p: int) -> np.ndarray:
    """Fixed probe vectors of the digest (seeded; entries in [-1, 1))."""
    return np.random.default_rng(20481).uniform(-1.0, 1.0, size=(p, NV))


def oracle_pass(out_path: str) -> None:
    c = full_scale_case()
    beta = np.asarray(c["coefs"])
    t0 = time.time()
    G, xtwz, s = po.pass_synth(c["kind"], c["row0"], c["n"], c["p"], c["seed"], c["family"], c["link"], beta=beta,
                               nthreads=os.cpu_count() or 8)
    np.savez(out_path, beta=beta, G=G, xtwz=xtwz, s=s)
    print(f"oracle pass at the full_scale coefficients: {time.time() - t0:.0f} s -> {out_path}", flush=True)


def lu_solve(G: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Breeze inv (the oracle's unblocked dgetrf + dgetri restatement), then inv * b (utils.scala:103-104)."""
    Gi = po.lu_inverse(G)
    x = np.zeros(len(b))
    for k in range(len(b)):  # inv * b summed over k in order, as the oracle's wls_solve (no FMA)
        x = x + Gi[:, k] * b[k]
    return x


def rel_elem(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300)))


def rel_norm(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def compare(engine_path: str, oracle_path: str) -> dict:
    e = np.load(engine_path)
    o = np.load(oracle_path)
    assert np.array_equal(e["beta"], o["beta"]), "engine and oracle passes at different beta"
    p = o["G"].shape[0]
    Ge = e["G"] if e["G"].ndim == 2 else unpack_lower(e["G"], p)
    Go, xo, xe = o["G"], o["xtwz"], e["xtwz"]
    # a) the Gram itself
    dG = np.abs(Ge - Go)
    a = {"gram_elementwise_max": float(np.max(dG / np.abs(Go))),
         "gram_normwise": float(np.linalg.norm(Ge - Go) / np.linalg.norm(Go)),
         "xtwz_elementwise_max": rel_elem(xe, xo),
         "deviance_rel": abs(float(e["s"][0]) - float(o["s"][0])) / abs(float(o["s"][0]))}
    # b) + c) the solves
    x_lu_e, x_lu_o = lu_solve(Ge, xe), lu_solve(Go, xo)
    x_chol_e = e["x_chol"]
    cond = float(np.linalg.cond(Go))
    res = {"case": CASE, "beta": "full_scale.json[gamma2048].coefs (the oracle's final coefficients)",
           "cond_gram": cond, "a_gram": a,
           "b_solve_chol_vs_lu_on_engine_gram": {"elementwise_max": rel_elem(x_chol_e, x_lu_e),
                                                  "normwise": rel_norm(x_chol_e, x_lu_e)},
           "c_gram_order_through_lu": {"elementwise_max": rel_elem(x_lu_e, x_lu_o), "normwise": rel_norm(x_lu_e, x_lu_o)},
           "total_engine_vs_oracle_solve": {"elementwise_max": rel_elem(x_chol_e, x_lu_o),
                                            "normwise": rel_norm(x_chol_e, x_lu_o)}}
    # the reference's own implementation spread on THIS matrix (the oracle's Gram): Breeze inv is LAPACK
    # dgetrf + dgetri as netlib-java binds it (here OpenBLAS through scipy), the oracle restates it
    # unblocked; a Cholesky solve is the engine's algorithm; the product inv * b in BLAS order
    import scipy.linalg as sl
    lu, piv = sl.lu_factor(Go)
    Gi_lapack, info = sl.lapack.dgetri(lu, piv)
    x_lapack = np.zeros(p)
    for k in range(p):
        x_lapack = x_lapack + Gi_lapack[:, k] * xo[k]
    x_chol_o = sl.cho_solve(sl.cho_factor(Go, lower=True), xo)
    res["reference_spread_on_oracle_gram"] = {
        "lapack_lu_vs_oracle_lu": {"elementwise_max": rel_elem(x_lapack, x_lu_o), "normwise": rel_norm(x_lapack, x_lu_o)},
        "lapack_lu_blas_product_vs_oracle_lu": {"elementwise_max": rel_elem(Gi_lapack @ xo, x_lu_o),
                                                "normwise": rel_norm(Gi_lapack @ xo, x_lu_o)},
        "lapack_cholesky_vs_oracle_lu": {"elementwise_max": rel_elem(x_chol_o, x_lu_o),
                                         "normwise": rel_norm(x_chol_o, x_lu_o)}}
    # the same in units of the solve's backward-error scale per coefficient, cond * eps * max|x| / |x_i|
    # (tests/test_gpu_configs.py wide_elementwise_ok bounds the engine by K_BOUND of these units)
    scale = cond * np.finfo(float).eps * np.max(np.abs(x_lu_o)) / np.abs(x_lu_o)
    res["K_units"] = {"reference_lapack_vs_oracle_lu": float(np.max(np.abs(x_lapack - x_lu_o) / np.abs(x_lu_o) / scale)),
                      "engine_chol_vs_oracle_lu": float(np.max(np.abs(x_chol_e - x_lu_o) / np.abs(x_lu_o) / scale))}
    if "fit_coefs" in e:
        fc = np.asarray(full_scale_case()["coefs"])
        res["K_units"]["engine_fit_vs_oracle_fit"] = float(np.max(np.abs(e["fit_coefs"] - fc) / np.abs(fc) / scale))
    if "x_lu_roc" in e:  # the engine's LU route (SGLM_WIDE_SOLVE=lu: rocSOLVER getrf + getri, inv * b in order)
        res["b_engine_lu_route_vs_oracle_lu_on_engine_gram"] = {"elementwise_max": rel_elem(e["x_lu_roc"], x_lu_e),
                                                                 "normwise": rel_norm(e["x_lu_roc"], x_lu_e)}
    if "fit_coefs" in e:
        c = full_scale_case()
        res["engine_fit_vs_oracle_fit"] = {"elementwise_max": rel_elem(e["fit_coefs"], c["coefs"]),
                                           "normwise": rel_norm(e["fit_coefs"], c["coefs"])}
    V = probe_vectors(p)
    digest = dict(beta=o["beta"], diag=np.diag(Go).copy(), GV=Go @ V, xtwz=xo, s=o["s"], x_lu_oracle=x_lu_o)
    return res, digest


def unpack_lower(packed: np.ndarray, p: int) -> np.ndarray:
    G = np.zeros((p, p))
    i, j = np.tril_indices(p)
    # packed row-major lower triangle: index i(i+1)/2 + j
    G[i, j] = packed[i * (i + 1) // 2 + j]
    G[j, i] = G[i, j]
    return G


def main(argv):
    build = os.path.join(HERE, "build")
    os.makedirs(build, exist_ok=True)
    oracle_path = os.path.join(build, "gram_split_oracle.npz")
    if argv[:1] == ["oracle"]:
        oracle_pass(oracle_path)
        return
    if argv[:1] == ["compare"]:
        res, digest = compare(argv[1], oracle_path)
        gold = os.path.join(ROOT, "tests", "golden")
        with open(os.path.join(gold, "gram_split_p2048.json"), "w") as fh:
            json.dump(res, fh, indent=1)
        np.savez_compressed(os.path.join(gold, "gram_split_p2048.npz"), **digest)
        print(json.dumps(res, indent=1))
        return
    print(__doc__)


if __name__ == "__main__":
    main(sys.argv[1:])
