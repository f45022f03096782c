"""ctypes binding for the CPU restatement (oracle/sglm_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, always as the checker (or the timed CPU baseline), never as the
thing measured or shipped.  The product package sparkglm_amd never imports this.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# SGLM_ORACLE_LIB selects another build of the same library (the sanitizer build, tools/asan_cpu.sh)
LIB_PATH = os.environ.get("SGLM_ORACLE_LIB") or os.path.join(HERE, "build", "libsglm_oracle.so")

FAMILIES = {"binomial": 0, "gaussian": 1, "poisson": 2, "gamma": 3}
LINKS = {"logit": 0, "probit": 1, "cloglog": 2, "identity": 3, "log": 4, "inverse": 5}
NS = 8


class _Opts(C.Structure):
    _fields_ = [("family", C.c_int), ("link", C.c_int), ("tol", C.c_double), ("max_iter", C.c_int),
                ("verbose", C.c_int), ("npart", C.c_int), ("nthreads", C.c_int), ("plain_sums", C.c_int)]


class _Pre(C.Structure):
    _fields_ = [("coefs", C.POINTER(C.c_double)), ("stderr_", C.POINTER(C.c_double)),
                ("deviance", C.c_double), ("null_deviance", C.c_double), ("pearson", C.c_double),
                ("loglik", C.c_double), ("iter", C.c_int), ("nrow", C.c_double), ("npart", C.c_int),
                ("dev_trace", C.POINTER(C.c_double)), ("max_trace", C.c_int)]


_lib = None


def build() -> None:
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        dp = C.POINTER(C.c_double)
        _lib.orc_fit_glm.argtypes = [dp, C.c_int64, C.c_int64, C.c_int64, dp, dp, dp, dp,
                                     C.POINTER(_Opts), C.POINTER(_Pre)]
        _lib.orc_fit_lm.argtypes = [dp, C.c_int64, C.c_int64, C.c_int64, dp, C.c_int, C.c_int,
                                    dp, dp, dp, dp, dp, dp, dp]
        _lib.orc_shard_partials.argtypes = [dp, C.c_int64, C.c_int64, C.c_int64, dp, dp, dp, dp,
                                            C.c_int, C.c_int, C.c_int, dp, C.c_double, C.c_double, dp]
        _lib.orc_lu_inverse.argtypes = [dp, C.c_int64]
        _lib.orc_fit_glm_synth.argtypes = [C.c_int, C.c_int64, C.c_int64, C.c_int64, C.c_uint64,
                                           C.POINTER(_Opts), C.POINTER(_Pre)]
        _lib.orc_synth_rows.argtypes = [C.c_int, C.c_int64, C.c_int64, C.c_int64, C.c_uint64, dp, dp, dp, dp]
        _lib.orc_pass_synth.argtypes = [C.c_int, C.c_int64, C.c_int64, C.c_int64, C.c_uint64, C.c_int, C.c_int,
                                        C.c_int, dp, C.c_double, C.c_int, dp, dp, dp]
        for f in ("orc_norm_cdf", "orc_norm_icdf", "orc_erfinv"):
            getattr(_lib, f).argtypes = [C.c_double]
            getattr(_lib, f).restype = C.c_double
    return _lib


def _ptr(a):
    if a is None:
        return None
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _col(a, n=None):
    if a is None:
        return None
    a = np.ascontiguousarray(a, dtype=np.float64).reshape(-1)
    if n is not None and a.shape[0] != n:
        raise ValueError("vector length mismatch")
    return a


@dataclass
class OraclePreGLM:
    coefs: np.ndarray
    stderr: np.ndarray
    deviance: float
    null_deviance: float
    pearson: float
    loglik: float
    iter: int
    nrow: float
    npart: int
    dev_trace: np.ndarray = field(default=None)


def fit_glm(X, y, family="binomial", link="logit", *, m=None, offset=None, prior=None, tol=1e-6,
            max_iter=0, npart=1, nthreads=1, verbose=False, max_trace=256) -> OraclePreGLM:
    X = np.asfortranarray(X, dtype=np.float64)
    n, p = X.shape
    y = _col(y, n)
    m, offset, prior = _col(m, n), _col(offset, n), _col(prior, n)
    coefs = np.zeros(p)
    se = np.zeros(p)
    trace = np.full(max_trace, np.nan)
    o = _Opts(FAMILIES[family], LINKS[link], tol, max_iter, int(verbose), npart, nthreads, 0)
    pre = _Pre(_ptr(coefs), _ptr(se), 0, 0, 0, 0, 0, 0, 0, _ptr(trace), max_trace)
    rc = lib().orc_fit_glm(_ptr(X), n, p, n, _ptr(y), _ptr(m), _ptr(offset), _ptr(prior),
                           C.byref(o), C.byref(pre))
    if rc != 0:
        raise RuntimeError(f"oracle orc_fit_glm failed rc={rc}")
    return OraclePreGLM(coefs, se, pre.deviance, pre.null_deviance, pre.pearson, pre.loglik,
                        pre.iter, pre.nrow, pre.npart, trace[: pre.iter + 1].copy())


def fit_glm_synth(kind, row0, n, p, seed, family="binomial", link="logit", *, tol=1e-6, max_iter=0, npart=1,
                  nthreads=8, verbose=False, max_trace=256, plain_sums=False) -> OraclePreGLM:
    """Streaming fit of rows [row0, row0+n) of the synthetic design (sparkglm_amd.synth), rows
    regenerated chunk by chunk every iteration (orc_fit_glm_synth): full-size parity without
    holding X in host RAM.  plain_sums: the reference's summation order for the deviance and the
    other scalars (per-partition plain running sums, partitions added in order; npart partitions)
    instead of compensated sums."""
    coefs, se, trace = np.zeros(p), np.zeros(p), np.full(max_trace, np.nan)
    o = _Opts(FAMILIES[family], LINKS[link], tol, max_iter, int(verbose), npart, nthreads, int(bool(plain_sums)))
    pre = _Pre(_ptr(coefs), _ptr(se), 0, 0, 0, 0, 0, 0, 0, _ptr(trace), max_trace)
    rc = lib().orc_fit_glm_synth(int(kind), int(row0), int(n), int(p), C.c_uint64(seed & (2**64 - 1)),
                                 C.byref(o), C.byref(pre))
    if rc != 0:
        raise RuntimeError(f"oracle orc_fit_glm_synth failed rc={rc}")
    return OraclePreGLM(coefs, se, pre.deviance, pre.null_deviance, pre.pearson, pre.loglik,
                        pre.iter, pre.nrow, pre.npart, trace[: pre.iter + 1].copy())


def pass_synth(kind, row0, n, p, seed, family, link, beta=None, mu0=0.0, mode=0, nthreads=8):
    """One pass of the streaming fit (orc_pass_synth) at beta: (X'WX p x p, X'Wz, scalars[8])."""
    G, xtwz, s = np.zeros((p, p), order="F"), np.zeros(p), np.zeros(NS)
    b = None if beta is None else np.ascontiguousarray(beta, dtype=np.float64)
    rc = lib().orc_pass_synth(int(kind), int(row0), int(n), int(p), C.c_uint64(seed & (2**64 - 1)),
                              FAMILIES[family], LINKS[link], int(mode), _ptr(b), float(mu0), int(nthreads),
                              G.ctypes.data_as(C.POINTER(C.c_double)), _ptr(xtwz), _ptr(s))
    if rc != 0:
        raise RuntimeError(f"oracle orc_pass_synth failed rc={rc}")
    return G, xtwz, s


def synth_rows(kind, row0, n, p, seed):
    """The oracle's C copy of the synthetic generator: (X (n x p, Fortran), y, offset, prior)."""
    X = np.empty((n, p), order="F")
    y, off, pr = np.empty(n), np.empty(n), np.empty(n)
    rc = lib().orc_synth_rows(int(kind), int(row0), int(n), int(p), C.c_uint64(seed & (2**64 - 1)),
                              X.ctypes.data_as(C.POINTER(C.c_double)), _ptr(y), _ptr(off), _ptr(pr))
    if rc != 0:
        raise RuntimeError("oracle orc_synth_rows failed")
    return X, y, (off if kind == 2 else None), (pr if kind == 2 else None)


def fit_lm(X, y, npart=1, nthreads=1):
    X = np.asfortranarray(X, dtype=np.float64)
    n, p = X.shape
    y = _col(y, n)
    coefs, xtxi, se = np.zeros(p), np.zeros((p, p), order="F"), np.zeros(p)
    sse, r2, f, sig = (C.c_double() for _ in range(4))
    rc = lib().orc_fit_lm(_ptr(X), n, p, n, _ptr(y), npart, nthreads, _ptr(coefs),
                          xtxi.ctypes.data_as(C.POINTER(C.c_double)), _ptr(se),
                          C.byref(sse), C.byref(r2), C.byref(f), C.byref(sig))
    if rc != 0:
        raise RuntimeError(f"oracle orc_fit_lm failed rc={rc}")
    return dict(coefs=coefs, xtxi=xtxi, stderr=se, sse=sse.value, r2=r2.value, fstat=f.value,
                sigma=sig.value)


def shard_partials(X, y, family, link, mode, beta=None, mu0=0.0, ybar=0.0, *, m=None, offset=None,
                   prior=None):
    """One shard's packed partials (mode: 0 irls, 1 init-single, 2 init-multi, 3 lm-gram, 4 lm-resid)."""
    X = np.asfortranarray(X, dtype=np.float64)
    n, p = X.shape
    y = _col(y, n)
    m, offset, prior = _col(m, n), _col(offset, n), _col(prior, n)
    out = np.zeros(p * (p + 1) // 2 + p + NS)
    b = None if beta is None else np.ascontiguousarray(beta, dtype=np.float64)
    rc = lib().orc_shard_partials(_ptr(X), n, p, n, _ptr(y), _ptr(m), _ptr(offset), _ptr(prior),
                                  FAMILIES[family], LINKS[link], int(mode), _ptr(b), mu0, ybar, _ptr(out))
    if rc != 0:
        raise RuntimeError(f"oracle orc_shard_partials failed rc={rc}")
    return out


def lu_inverse(A):
    A = np.asfortranarray(A, dtype=np.float64).copy(order="F")
    rc = lib().orc_lu_inverse(A.ctypes.data_as(C.POINTER(C.c_double)), A.shape[0])
    if rc != 0:
        raise np.linalg.LinAlgError("singular")
    return A
