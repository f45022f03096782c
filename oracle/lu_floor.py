"""The conditioning floor of configs[3] (gamma/inverse, p = 2048): how far apart two correct
implementations of the reference's own solve land on the SAME X'WX.

TEST INFRASTRUCTURE / EVIDENCE ONLY (never imported by sparkglm_amd).

The reference solves every IRLS step with Breeze `inv` -- LAPACK dgetrf + dgetri through
netlib-java -- and `coefs = XtWXi * XtWy`, `stdErr = sqrt(diag(XtWXi))` (utils.scala:103-105,
134-136).  Which LAPACK runs is decided at run time by netlib-java (F2J reference LAPACK,
the system's native LAPACK, OpenBLAS, MKL ...), and each of those blocks dgetrf / dgetri /
dgemm differently, so the reference's own coefficients are defined only up to that
implementation's rounding, ~cond(X'WX) * eps relative.  This script measures the spread on the
oracle's X'WX of the last solve of a configs[3]-shaped fit:

  oracle   orc_lu_inverse (unblocked dgetrf + dgetri restated, oracle/sglm_oracle.c:234)
  lapack   scipy.linalg.lapack dgetrf + dgetri (OpenBLAS's blocked LAPACK: what netlib-java
           binds when a native LAPACK is installed) then inv * b as the reference does
  lapack_solve  dgetrs instead of the explicit inverse (same factor)
  chol     dpotrf + dpotrs (the engine's round-2 wide solve)
  gram_blas  the same fit's X'WX re-summed in another order (numpy/BLAS X.T @ (w X)), solved by
           the oracle's LU: the summation-order part every engine differs from any other by

and prints, for each, the largest elementwise relative coefficient / stdErr difference against
the oracle, the norm-wise one, and cond(X'WX).

  python oracle/lu_floor.py [--n 6000] [--p 2048] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import scipy.linalg.lapack as lapack

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pyoracle as po  # noqa: E402


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b) / np.abs(b)))


def nrel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / np.max(np.abs(b)))


def unpack(packed, p):
    tri = p * (p + 1) // 2
    A = np.zeros((p, p))
    # packed lower triangle, row-major: (i, j) for j <= i
    r = np.repeat(np.arange(p), np.arange(1, p + 1))
    c = np.arange(tri) - r * (r + 1) // 2
    A[r, c] = packed[:tri]
    A[c, r] = packed[:tri]
    return A, packed[tri:tri + p].copy()


def lapack_inv(A):
    lu, piv, info = lapack.dgetrf(A)
    assert info == 0
    inv, info = lapack.dgetri(lu, piv)
    assert info == 0
    return inv, lu, piv


def run(n=6000, p=2048, row0=777, seed=4, nthreads=8):
    t0 = time.time()
    X, y, _, _ = po.synth_rows(3, row0, n, p, seed)
    full = po.fit_glm(X, y, "gamma", "inverse", nthreads=nthreads)
    k = full.iter
    # beta_{k-1}: the coefficients whose weights build the X'WX of the k-th (last) solve
    if k >= 2:
        prev = po.fit_glm(X, y, "gamma", "inverse", nthreads=nthreads, max_iter=k - 1)
        packed = po.shard_partials(X, y, "gamma", "inverse", 0, beta=prev.coefs)
    else:
        packed = po.shard_partials(X, y, "gamma", "inverse", 1, mu0=float(np.mean(y)))
    A, b = unpack(packed, p)
    out = {"n": n, "p": p, "iter": k, "cond": float(np.linalg.cond(A))}

    Ai = po.lu_inverse(A)
    c_orc = Ai @ b
    se_orc = np.sqrt(np.diag(Ai))
    out["oracle_reproduces_fit"] = {"coefs": rel(c_orc, full.coefs), "stderr": rel(se_orc, full.stderr)}

    cands = {}
    inv, lu, piv = lapack_inv(A)
    cands["lapack"] = (inv @ b, np.sqrt(np.diag(inv)))
    xs, info = lapack.dgetrs(lu, piv, b)
    cands["lapack_solve"] = (xs, np.sqrt(np.diag(inv)))
    L, info = lapack.dpotrf(A, lower=1)
    assert info == 0
    xc, info = lapack.dpotrs(L, b, lower=1)
    Li, info = lapack.dpotri(L, lower=1)
    Li = np.tril(Li) + np.tril(Li, -1).T
    cands["chol"] = (xc, np.sqrt(np.diag(Li)))
    # the same X'WX summed in another order (BLAS dgemm): w from the oracle's own weights
    if k >= 2:
        eta = X @ prev.coefs
        mu = 1.0 / eta
        w = 1.0 / (mu * mu * (1.0 / (mu * mu)) ** 2)
    else:
        mu0 = float(np.mean(y))
        w = np.full(n, 1.0 / (mu0 * mu0 * (1.0 / (mu0 * mu0)) ** 2))
    A2 = X.T @ (w[:, None] * X)
    A2 = 0.5 * (A2 + A2.T)
    out["gram_blas_vs_oracle_gram"] = nrel(A2, A)
    Ai2 = po.lu_inverse(A2)
    cands["gram_blas"] = (Ai2 @ b, np.sqrt(np.diag(Ai2)))

    absb = np.abs(c_orc)
    small = np.argsort(absb)[:5]
    for name, (c, se) in cands.items():
        out[name] = {"coefs_rel": rel(c, c_orc), "coefs_nrel": nrel(c, c_orc), "stderr_rel": rel(se, se_orc),
                     "worst_coef": int(np.argmax(np.abs(c - c_orc) / np.abs(c_orc))),
                     "smallest_coefs_rel": [float(abs(c[i] - c_orc[i]) / abs(c_orc[i])) for i in small]}
    out["smallest_abs_coefs"] = [float(absb[i]) for i in small]
    out["max_abs_coef"] = float(absb.max())
    out["seconds"] = round(time.time() - t0, 1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=6000)
    ap.add_argument("--p", type=int, default=2048)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    out = run(a.n, a.p)
    s = json.dumps(out, indent=1)
    print(s)
    if a.json:
        with open(a.json, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
