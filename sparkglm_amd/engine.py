"""Python handle over the C ABI: one `Engine` per HIP device (one per rank).

This is plumbing around libsglm_hip.so; every fit runs in the C++ driver and the gfx950
kernels.  See include/sglm.h for the contract of each call.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L


@dataclass
class FitGLM:
    """PreGLM (GLM.scala:25-33) plus the deviance trace."""
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


@dataclass
class FitLM:
    """PreLM (LM.scala:10-14) plus LM.fit's stdErr and sigma (LM.scala:260-263)."""
    coefs: np.ndarray
    xtxi: np.ndarray
    stderr: np.ndarray
    sse: float
    r2: float
    fstat: float
    sigma: float
    nrow: float
    npart: int


def _vec(a, n):
    if a is None:
        return None
    a = np.ascontiguousarray(a, dtype=np.float64).reshape(-1)
    if a.shape[0] != n:
        raise L.IllegalArgumentException("requirement failed: The two DataFrames must have the same number of rows")
    return a


def glm_opts(family="binomial", link="logit", tol=1e-6, verbose=False, max_iter=0, init="single", npart=0):
    fam = family.lower()
    if fam not in L.FAMILIES:
        raise L.IllegalArgumentException(f"requirement failed: unknown family {family!r}")
    if link not in L.LINKS:
        raise L.IllegalArgumentException(f"requirement failed: unknown link {link!r}")
    return L.GlmOpts(L.FAMILIES[fam], L.LINKS[link], float(tol), int(bool(verbose)), int(max_iter),
                     L.INIT_MULTIPLE if init == "multiple" else L.INIT_SINGLE, int(npart))


class Engine:
    """One HIP device holding one row shard of the design in HBM (SURVEY 8(b)'s constructor
    sglm_create(const int* devs, int ndev = 1)) -- or, with `devices=[...]`, the group handle over
    those devices (sglm_create_multi: row shards per device, one RCCL group all-reduce per
    iteration, for one listed device too; a device listed twice shares the card and sums on the
    host)."""

    def __init__(self, device: int = 0, devices=None):
        self._lib = L.load()
        h = C.c_void_p()
        if devices is not None:
            devs = (C.c_int * len(devices))(*[int(d) for d in devices])
            L.check(self._lib.sglm_create_multi(devs, len(devices), C.byref(h)), "sglm_create_multi")
            device = int(devices[0])
        else:
            one = (C.c_int * 1)(int(device))
            L.check(self._lib.sglm_create(one, 1, C.byref(h)), "sglm_create")
        self._h = h
        self.device = device
        self.devices = list(devices) if devices is not None else [device]
        self.n = 0
        self.p = 0
        self._comm_keep = None

    # ---- lifecycle ----
    def close(self):
        if getattr(self, "_h", None):
            self._lib.sglm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- data ----
    def set_data(self, X, y, m=None, offset=None, prior=None):
        X = np.asfortranarray(X, dtype=np.float64)
        if X.ndim != 2:
            raise L.IllegalArgumentException("requirement failed: X must be a matrix")
        n, p = X.shape
        y, m, offset, prior = _vec(y, n), _vec(m, n), _vec(offset, n), _vec(prior, n)
        L.check(self._lib.sglm_set_data(self._h, L.ptr(X), n, p, n, L.ptr(y), L.ptr(m), L.ptr(offset),
                                        L.ptr(prior)), "sglm_set_data")
        self.n, self.p = n, p
        return self

    def reserve(self, n: int, p: int, m=False, offset=False, prior=False):
        """Allocate the resident shard; rows then arrive by set_rows (partition-wise ingest)."""
        L.check(self._lib.sglm_reserve(self._h, int(n), int(p), int(bool(m)), int(bool(offset)), int(bool(prior))),
                "sglm_reserve")
        self.n, self.p = int(n), int(p)
        return self

    def set_rows(self, row0: int, X, y, m=None, offset=None, prior=None):
        """Rows [row0, row0 + len(y)) of the reserved shard (one Spark partition's block)."""
        X = np.asfortranarray(X, dtype=np.float64)
        nr = X.shape[0]
        y, m, offset, prior = _vec(y, nr), _vec(m, nr), _vec(offset, nr), _vec(prior, nr)
        L.check(self._lib.sglm_set_rows(self._h, int(row0), nr, L.ptr(X), max(nr, 1), L.ptr(y), L.ptr(m),
                                        L.ptr(offset), L.ptr(prior)), "sglm_set_rows")
        return self

    def set_data_device(self, X, y, m=None, offset=None, prior=None):
        """Torch tensors already on this engine's device: X (n, p) column-major (stride(0) == 1,
        e.g. X.t().contiguous().t()), y / m / offset / prior contiguous length-n vectors, all
        float64.  The engine copies n doubles from every pointer, so anything else is refused
        here rather than read past its allocation."""
        import torch
        if X.dim() != 2:
            raise L.IllegalArgumentException("requirement failed: X must be a matrix")
        n, p = X.shape
        ldx = X.stride(1)
        dev = torch.device("cuda", self.device)

        def _ok(t, what):
            if t.dtype != torch.float64:
                raise L.IllegalArgumentException(f"requirement failed: {what} must be float64, got {t.dtype}")
            if not t.is_cuda or t.device != dev:
                raise L.IllegalArgumentException(f"requirement failed: {what} must live on {dev}, got {t.device}")

        _ok(X, "X")
        if X.stride(0) != 1 or (p > 1 and ldx < n):
            raise L.IllegalArgumentException("requirement failed: X must be column-major on device (stride(0) == 1, "
                                             "leading dimension >= n)")
        for t, what in ((y, "y"), (m, "m"), (offset, "offset"), (prior, "prior")):
            if t is None:
                continue
            _ok(t, what)
            if tuple(t.shape) not in ((n,), (n, 1)) or (n > 1 and t.stride(0) != 1):
                raise L.IllegalArgumentException(f"requirement failed: {what} must be a contiguous vector of "
                                                 f"length {n}")
        ldx = max(ldx, n) if p == 1 else ldx
        g = lambda t: None if t is None else C.c_void_p(t.data_ptr())
        L.check(self._lib.sglm_set_data_device(self._h, g(X), n, p, ldx, g(y), g(m), g(offset), g(prior)),
                "sglm_set_data_device")
        self.n, self.p = n, p
        return self

    def synth(self, kind: int, row0: int, n: int, p: int, seed: int, procedural: bool = False):
        """Rows [row0, row0+n) of the seeded synthetic design generated in HBM.  procedural=True
        stores y (+ offset / prior) only and regenerates X inside the kernels (wide path)."""
        fn = self._lib.sglm_synth_procedural if procedural else self._lib.sglm_synth
        L.check(fn(self._h, int(kind), int(row0), int(n), int(p), C.c_uint64(seed & (2**64 - 1))),
                "sglm_synth_procedural" if procedural else "sglm_synth")
        self.n, self.p = n, p
        return self

    def get_data(self):
        X = np.empty((self.n, self.p), order="F")
        y, m, off, pr = (np.empty(self.n) for _ in range(4))
        L.check(self._lib.sglm_get_data(self._h, L.ptr(X), L.ptr(y), L.ptr(m), L.ptr(off), L.ptr(pr)))
        return X, y, m, off, pr

    # ---- communicators ----
    def set_comm(self, fn, on_device: bool, rank=None):
        """fn(buf_ptr:int, count:int, stream:int, on_device:bool) -> None, sums in place.  With
        `rank` (this process's rank in fn's group) the scalars are summed in rank order with
        compensation (sglm_set_comm_rank)."""
        def _cb(ctx, buf, count, stream, dev):
            try:
                fn(C.cast(buf, C.c_void_p).value, int(count), stream, bool(dev))
                return 0
            except Exception:  # an exception cannot cross the C frame
                import traceback
                traceback.print_exc()
                return 1
        cb = L.ALLREDUCE_FN(_cb)
        self._comm_keep = cb
        L.check(self._lib.sglm_set_comm(self._h, cb, None, int(bool(on_device))), "sglm_set_comm")
        if rank is not None:
            L.check(self._lib.sglm_set_comm_rank(self._h, int(rank)), "sglm_set_comm_rank")

    def set_comm_local(self, rank):
        """Join an in-process communicator (distributed.LocalComm(n).rank(r)): host threads of
        one process, one engine each."""
        self._comm_keep = rank
        L.check(self._lib.sglm_set_comm(self._h, rank.comm.fn, C.c_void_p(rank.ctx), 0), "sglm_set_comm")

    def set_comm_rccl(self, nranks: int, rank: int, unique_id: bytes):
        buf = C.create_string_buffer(bytes(unique_id), 128)
        L.check(self._lib.sglm_set_comm_rccl(self._h, int(nranks), int(rank), buf), "sglm_set_comm_rccl")

    @staticmethod
    def rccl_unique_id() -> bytes:
        lib = L.load()
        buf = C.create_string_buffer(128)
        L.check(lib.sglm_rccl_unique_id(buf), "sglm_rccl_unique_id")
        return buf.raw

    # ---- fits ----
    def fit_glm(self, family="binomial", link="logit", tol=1e-6, verbose=False, max_iter=0, init="single",
                npart=0, max_trace=512) -> FitGLM:
        o = glm_opts(family, link, tol, verbose, max_iter, init, npart)
        coefs, se = np.zeros(self.p), np.zeros(self.p)
        trace = np.full(max_trace, np.nan)
        pre = L.PreGLM(L.ptr(coefs), L.ptr(se), 0, 0, 0, 0, 0, 0, 0, L.ptr(trace), max_trace)
        L.check(self._lib.sglm_fit_glm(self._h, C.byref(o), C.byref(pre)), "sglm_fit_glm")
        return FitGLM(coefs, se, pre.deviance, pre.null_deviance, pre.pearson, pre.loglik, pre.iter, pre.nrow,
                      pre.npart, trace[: pre.iter + 1].copy())

    def fit_lm(self) -> FitLM:
        p = self.p
        coefs, se, xtxi = np.zeros(p), np.zeros(p), np.zeros((p, p), order="F")
        pre = L.PreLM(L.ptr(coefs), xtxi.ctypes.data_as(L.dp), L.ptr(se), 0, 0, 0, 0, 0, 0)
        L.check(self._lib.sglm_fit_lm(self._h, C.byref(pre)), "sglm_fit_lm")
        return FitLM(coefs, xtxi, se, pre.sse, pre.r2, pre.fstat, pre.sigma, pre.nrow, pre.npart)

    def irls_pass(self, beta=None, mu0=0.0, family="binomial", link="logit", init="single"):
        o = glm_opts(family, link, init=init)
        p = self.p
        gram, xtwz, s = np.zeros((p, p), order="F"), np.zeros(p), np.zeros(L.NS)
        b = None if beta is None else np.ascontiguousarray(beta, dtype=np.float64)
        L.check(self._lib.sglm_irls_pass(self._h, C.byref(o), L.ptr(b), float(mu0), gram.ctypes.data_as(L.dp),
                                         L.ptr(xtwz), L.ptr(s)), "sglm_irls_pass")
        return gram, xtwz, s

    def irls_step(self, beta, family="binomial", link="logit"):
        """SURVEY 8(b)'s test-level step: X'WX, X'Wz and the deviance at beta."""
        o = glm_opts(family, link)
        p = self.p
        xtwx, xtwz, dev = np.zeros((p, p), order="F"), np.zeros(p), C.c_double()
        b = np.ascontiguousarray(beta, dtype=np.float64)
        L.check(self._lib.sglm_irls_step(self._h, C.byref(o), L.ptr(b), xtwx.ctypes.data_as(L.dp), L.ptr(xtwz),
                                         C.byref(dev)), "sglm_irls_step")
        return xtwx, xtwz, dev.value

    def irls_iterations(self, beta, iters, family="binomial", link="logit"):
        o = glm_opts(family, link)
        b = np.ascontiguousarray(beta, dtype=np.float64).copy()
        dev = C.c_double()
        L.check(self._lib.sglm_irls_iterations(self._h, C.byref(o), L.ptr(b), int(iters), C.byref(dev)),
                "sglm_irls_iterations")
        return b, dev.value

    def predict(self, beta, add_offset=False):
        b = np.ascontiguousarray(beta, dtype=np.float64)
        out = np.empty(self.n)
        L.check(self._lib.sglm_predict(self._h, L.ptr(b), int(bool(add_offset)), L.ptr(out)), "sglm_predict")
        return out

    def predict_glm(self, beta, family="binomial", link="logit", type="response", add_offset=True):
        """Fitted values of the resident rows on the link or response scale."""
        o = glm_opts(family, link)
        b = np.ascontiguousarray(beta, dtype=np.float64).reshape(-1)
        out = np.empty(self.n)
        L.check(self._lib.sglm_predict_glm(self._h, L.ptr(b), o.family, o.link, _ptype(type), int(bool(add_offset)),
                                           L.ptr(out)), "sglm_predict_glm")
        return out

    def predict_new(self, X, beta, family="gaussian", link="identity", type="link", offset=None, m=None):
        """Score new rows without touching the resident shard (LM.predict; GLM response scale)."""
        o = glm_opts(family, link)
        X = np.asfortranarray(X, dtype=np.float64)
        if X.ndim != 2:
            raise L.IllegalArgumentException("requirement failed: X must be a matrix")
        n, p = X.shape
        b = np.ascontiguousarray(beta, dtype=np.float64).reshape(-1)
        if b.shape[0] != p:
            raise L.IllegalArgumentException(f"requirement failed: Dimension mismatch: X has {p} columns, "
                                             f"beta {b.shape[0]} rows")
        offset, m = _vec(offset, n), _vec(m, n)
        out = np.empty(n)
        L.check(self._lib.sglm_predict_new(self._h, L.ptr(X), n, p, max(n, 1), L.ptr(b), L.ptr(offset), L.ptr(m),
                                           o.family, o.link, _ptype(type), L.ptr(out)), "sglm_predict_new")
        return out

    def stats(self) -> dict:
        s = L.Stats()
        L.check(self._lib.sglm_get_stats(self._h, C.byref(s)))
        d = {k: getattr(s, k) for k, _ in L.Stats._fields_}
        d["comm_path_name"] = L.COMM_PATHS.get(d["comm_path"], "?")
        d["solve_path_name"] = L.SOLVE_PATHS.get(d["solve_path"], "?")
        d["pass_kernel_name"] = s.pass_kernel_name.decode()
        d["pass_kernel_kind"] = L.PASS_KERNELS.get(d["pass_kernel"], "?")
        return d

    def reset_stats(self):
        L.check(self._lib.sglm_reset_stats(self._h))


def _ptype(t) -> int:
    if t not in ("link", "response"):
        raise L.IllegalArgumentException(f"requirement failed: type must be 'link' or 'response', got {t!r}")
    return L.PREDICT_RESPONSE if t == "response" else L.PREDICT_LINK


def device_count() -> int:
    lib = L.load()
    c = C.c_int()
    rc = lib.sglm_device_count(C.byref(c))
    return c.value if rc == 0 else 0
