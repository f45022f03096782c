"""Row sharding and communicators for multi-GPU fits (one process per GPU).

The reference partitions rows across Spark tasks and sums the per-partition normal
equations with ml-matrix treeReduce (utils.scala:110-126).  Here each rank keeps its
contiguous row shard resident in its own HBM and the engine all-reduces one packed
buffer per IRLS iteration (lower-triangular X'WX | X'Wz | scalars):

  * natively over RCCL/xGMI (Engine.set_comm_rccl; unique id broadcast by the caller), or
  * through any torch.distributed process group (torch_allreduce): RCCL ("nccl") on
    device buffers, or gloo on host buffers.

`fit_glm_external` / `fit_lm_external` run the engine's C++ driver over caller-produced
partials (sglm_fit_*_external) -- the same driver, solve and convergence logic as a GPU
fit, usable wherever the partial sums come from elsewhere.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L
from .engine import FitGLM, FitLM, glm_opts


def shard_range(n_global: int, world: int, rank: int):
    """Rows [lo, hi) of `rank`: Spark's ParallelCollectionRDD slicing, [r*n/G, (r+1)*n/G)."""
    return (rank * n_global) // world, ((rank + 1) * n_global) // world


class _DeviceBuffer:
    def __init__(self, ptr: int, count: int):
        self.__cuda_array_interface__ = {"shape": (count,), "typestr": "<f8", "data": (ptr, False),
                                         "version": 3, "strides": None}


def torch_allreduce(group=None):
    """All-reduce callback over a torch.distributed group (sum, fp64, in place)."""
    import torch
    import torch.distributed as dist

    def fn(ptr: int, count: int, stream, on_device: bool):
        if on_device:
            t = torch.as_tensor(_DeviceBuffer(ptr, count), device="cuda")
            dist.all_reduce(t, group=group)
            torch.cuda.synchronize()
        else:
            a = np.ctypeslib.as_array((C.c_double * count).from_address(ptr))
            t = torch.from_numpy(a)
            dist.all_reduce(t, group=group)
    return fn


class LocalComm:
    """The library's in-process communicator (sglm_local_comm): N host threads in one process,
    one handle (or external fit) each -- the thread-pool alternative to sglm_create_multi.  The
    sum runs in rank order inside the library, so every rank gets bitwise the same buffer."""

    def __init__(self, nranks: int):
        self._lib = L.load()
        c = C.c_void_p()
        L.check(self._lib.sglm_local_comm_create(int(nranks), C.byref(c)), "sglm_local_comm_create")
        self._c = c
        self.nranks = nranks
        # the C function itself (no Python frame on the reduction path)
        self.fn = L.ALLREDUCE_FN(C.cast(self._lib.sglm_local_allreduce, C.c_void_p).value)

    def rank(self, r: int) -> "LocalRank":
        ctx = self._lib.sglm_local_comm_rank(self._c, int(r))
        if not ctx:
            raise L.IllegalArgumentException(f"requirement failed: rank {r} of {self.nranks}")
        return LocalRank(self, ctx)

    def close(self):
        if getattr(self, "_c", None):
            self._lib.sglm_local_comm_destroy(self._c)
            self._c = None


class LocalRank:
    def __init__(self, comm: LocalComm, ctx: int):
        self.comm, self.ctx = comm, ctx


def _comm_args(allreduce):
    """(C all-reduce function, its context) for a Python callable, a LocalRank, or None."""
    if isinstance(allreduce, LocalRank):
        return allreduce.comm.fn, C.c_void_p(allreduce.ctx)
    return _allreduce_cb(allreduce), None


def _allreduce_cb(fn):
    if fn is None:
        return L.ALLREDUCE_FN(lambda ctx, buf, count, stream, dev: 0)

    def _cb(ctx, buf, count, stream, dev):
        try:
            fn(C.cast(buf, C.c_void_p).value, int(count), stream, bool(dev))
            return 0
        except Exception:
            import traceback
            traceback.print_exc()
            return 1
    return L.ALLREDUCE_FN(_cb)


class _ExternalBackend:
    """Adapts Python callables to the C `sglm_backend` vtable.

    local_sums() -> (sum_y, n_local);  partials(mode, beta|None, mu0, ybar) -> packed array.
    """

    def __init__(self, p: int, local_sums, partials):
        self.p = p
        self.packed_len = p * (p + 1) // 2 + p + L.NS

        def _sums(ctx, out):
            try:
                s, n = local_sums()
                out[0], out[1] = float(s), float(n)
                return 0
            except Exception:
                import traceback
                traceback.print_exc()
                return 1

        def _pass(ctx, mode, beta, mu0, ybar, packed):
            try:
                b = None if not beta else np.ctypeslib.as_array(beta, shape=(p,)).copy()
                res = np.ascontiguousarray(partials(int(mode), b, float(mu0), float(ybar)), dtype=np.float64)
                if res.size != self.packed_len:  # the C side owns exactly packed_len doubles
                    raise ValueError(f"partials() returned {res.size} doubles, the packed wire format of "
                                     f"p = {p} holds {self.packed_len}")
                C.memmove(packed, res.ctypes.data, res.nbytes)
                return 0
            except Exception:
                import traceback
                traceback.print_exc()
                return 1

        self._keep = (L.LOCAL_SUMS_FN(_sums), L.PASS_FN(_pass))
        self.struct = L.Backend(None, p, self._keep[0], self._keep[1])


def fit_glm_external(p, local_sums, partials, allreduce=None, family="binomial", link="logit", tol=1e-6,
                     max_iter=0, init="single", npart=0, max_trace=512) -> FitGLM:
    lib = L.load()
    be = _ExternalBackend(p, local_sums, partials)
    cb, ctx = _comm_args(allreduce)
    o = glm_opts(family, link, tol, False, max_iter, init, npart)
    coefs, se, trace = np.zeros(p), np.zeros(p), np.full(max_trace, np.nan)
    pre = L.PreGLM(L.ptr(coefs), L.ptr(se), 0, 0, 0, 0, 0, 0, 0, L.ptr(trace), max_trace)
    L.check(lib.sglm_fit_glm_external(C.byref(be.struct), cb, ctx, C.byref(o), C.byref(pre)),
            "sglm_fit_glm_external")
    return FitGLM(coefs, se, pre.deviance, pre.null_deviance, pre.pearson, pre.loglik, pre.iter, pre.nrow,
                  pre.npart, trace[: pre.iter + 1].copy())


def fit_lm_external(p, local_sums, partials, allreduce=None) -> FitLM:
    lib = L.load()
    be = _ExternalBackend(p, local_sums, partials)
    cb, ctx = _comm_args(allreduce)
    coefs, se, xtxi = np.zeros(p), np.zeros(p), np.zeros((p, p), order="F")
    pre = L.PreLM(L.ptr(coefs), xtxi.ctypes.data_as(L.dp), L.ptr(se), 0, 0, 0, 0, 0, 0)
    L.check(lib.sglm_fit_lm_external(C.byref(be.struct), cb, ctx, C.byref(pre)), "sglm_fit_lm_external")
    return FitLM(coefs, xtxi, se, pre.sse, pre.r2, pre.fstat, pre.sigma, pre.nrow, pre.npart)
