"""Seeded synthetic designs, bit-identical to the engine's device generator.

The same counter-based generator runs on the GPU (sglm_synth, kernels.hip synth_kernel)
so that a test can regenerate any rank's shard on the host: X[i, j] for global row i is a
pure function of (seed, i, j), computed with integer hashing (splitmix64) and IEEE
multiply/add only (no FMA contraction, no libm).

  column 0: intercept 1.0
  column j>0: (2u - 1) / sqrt(p),   u = (splitmix64(sm(seed) + i*p + j) >> 11) * 2^-53
  eta* = sum_j x_ij b_j,  b_0 = -0.25,  b_j = 0.5 * ((j mod 5) - 2)   (sequential sum)
  kind 0 (logit design):   y = [u_y < clamp(0.5 + 0.25 eta*, 0.02, 0.98)]
  kind 1 (gaussian):       y = eta* + (2 u_y - 1)
  kind 2 (poisson counts): y = floor(u_y * 2 * max(1 + 0.5 eta*, 0.1)),
                           offset = 0.1 (2 u_o - 1),  prior = 0.5 + u_p
  kind 3 (gamma, inverse link): column j>0 is (0.5 + u) / sqrt(p) (positive), b_0 = 1,
                           b_j = 0.1 ((j mod 5) + 1), y = (0.25 + 1.5 u_y) / eta*  (> 0)
"""
from __future__ import annotations

import numpy as np

M64 = (1 << 64) - 1
_GOLD = np.uint64(0x9E3779B97F4A7C15)
_C1 = np.uint64(0xBF58476D1CE4E5B9)
_C2 = np.uint64(0x94D049BB133111EB)


def splitmix64(x):
    """Vectorised splitmix64 finaliser over uint64 arrays (wrapping arithmetic)."""
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + _GOLD
        z = (z ^ (z >> np.uint64(30))) * _C1
        z = (z ^ (z >> np.uint64(27))) * _C2
    return z ^ (z >> np.uint64(31))


def _sm_scalar(x: int) -> int:
    return int(splitmix64(np.uint64(x & M64)))


def unif(keys):
    return (splitmix64(keys) >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


def beta_star(p: int, kind: int = 0) -> np.ndarray:
    if kind == 3:
        b = np.array([0.1 * ((j % 5) + 1) for j in range(p)], dtype=np.float64)
        b[0] = 1.0
        return b
    b = np.array([0.5 * ((j % 5) - 2) for j in range(p)], dtype=np.float64)
    b[0] = -0.25
    return b


def generate(kind: int, row0: int, n: int, p: int, seed: int):
    """Rows [row0, row0+n) of the synthetic design: (X (n x p, Fortran order), y, offset, prior)."""
    kx = _sm_scalar(seed)
    ky = _sm_scalar(seed ^ 0x5555555555555555)
    ko = _sm_scalar(seed ^ 0x3333333333333333)
    kp = _sm_scalar(seed ^ 0x0F0F0F0F0F0F0F0F)
    gi = np.arange(row0, row0 + n, dtype=np.uint64)
    scale = 1.0 / np.sqrt(np.float64(p))
    X = np.empty((n, p), dtype=np.float64, order="F")
    bs = beta_star(p, kind)
    eta = np.zeros(n, dtype=np.float64)
    with np.errstate(over="ignore"):
        base = np.uint64(kx) + gi * np.uint64(p)
        for j in range(p):
            if j == 0:
                x = np.ones(n, dtype=np.float64)
            elif kind == 3:
                x = (0.5 + unif(base + np.uint64(j))) * scale
            else:
                x = (2.0 * unif(base + np.uint64(j)) - 1.0) * scale
            X[:, j] = x
            prod = x * bs[j]
            eta = eta + prod
        u = unif(np.uint64(ky) + gi)
        offset = prior = None
        if kind == 0:
            pr = np.clip(0.5 + 0.25 * eta, 0.02, 0.98)
            y = (u < pr).astype(np.float64)
        elif kind == 1:
            y = eta + (2.0 * u - 1.0)
        elif kind == 2:
            lam = np.maximum(1.0 + 0.5 * eta, 0.1)
            y = np.floor(u * 2.0 * lam)
            offset = (2.0 * unif(np.uint64(ko) + gi) - 1.0) * 0.1
            prior = 0.5 + unif(np.uint64(kp) + gi)
        elif kind == 3:
            y = (0.25 + 1.5 * u) / eta
        else:
            raise ValueError("kind must be 0, 1, 2 or 3")
    return X, y, offset, prior
