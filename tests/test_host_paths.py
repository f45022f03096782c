"""Host-side paths of the C-ABI library that need no GPU: the in-process communicator (N host
threads, one fit each -- a JVM driver's thread pool), the external backend's wire-format check,
the multi-device handle's refusal without a device, and the solve on ill-conditioned designs.
Partials come from the oracle (the checker)."""
import ctypes as C
import threading

import numpy as np
import pytest

import pyoracle as po
from conftest import check_fit, rel
from sparkglm_amd import _lib as L
from sparkglm_amd import distributed as D


def _thread_fits(X, y, fam, link, world, kw, lm=False):
    comm = D.LocalComm(world)
    res, errs = {}, []

    def run(r):
        try:
            lo, hi = D.shard_range(len(y), world, r)
            Xs, ys = np.asfortranarray(X[lo:hi]), y[lo:hi]
            kws = {k: (None if v is None else v[lo:hi]) for k, v in kw.items()}
            sums = lambda: (ys.sum(), len(ys))
            if lm:
                part = lambda mode, b, mu0, ybar: po.shard_partials(Xs, ys, "gaussian", "identity", mode, b, mu0, ybar)
                res[r] = D.fit_lm_external(X.shape[1], sums, part, allreduce=comm.rank(r))
            else:
                part = lambda mode, b, mu0, ybar: po.shard_partials(Xs, ys, fam, link, mode, b, mu0, ybar, **kws)
                res[r] = D.fit_glm_external(X.shape[1], sums, part, allreduce=comm.rank(r), family=fam, link=link,
                                            init="multiple")
        except Exception as e:  # pragma: no cover - surfaced below
            errs.append(e)

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    comm.close()
    assert not errs, errs
    return res


@pytest.mark.parametrize("name,world", [("logit", 3), ("poisson_offset_prior", 4), ("probit", 2)])
def test_threads_in_one_process_equal_partitioned_fit(golden, name, world):
    """one host process driving N shards from N threads (one handle each), joined by
    the library's in-process all-reduce, gives the partitioned reference fit on every thread."""
    c = golden[name]
    fam, link = (str(v) for v in c["meta"][:2])
    kw = {"offset": c.get("offset"), "prior": c.get("prior"), "m": c.get("m")}
    res = _thread_fits(c["X"], c["y"], fam, link, world, kw)
    ref = po.fit_glm(c["X"], c["y"], fam, link, npart=world, nthreads=world, **kw)
    for r in range(world):
        f = res[r]
        assert f.iter == ref.iter and f.npart == world and f.nrow == len(c["y"])
        assert rel(f.coefs, ref.coefs) < 1e-10 and rel(f.stderr, ref.stderr) < 1e-10
        assert rel([f.deviance, f.null_deviance, f.pearson, f.loglik],
                   [ref.deviance, ref.null_deviance, ref.pearson, ref.loglik]) < 1e-10
        np.testing.assert_array_equal(f.coefs, res[0].coefs)  # rank-order sums: bitwise equal


def test_threads_lm(golden):
    c = golden["gaussian"]
    res = _thread_fits(c["X"], c["y"], None, None, 3, {}, lm=True)
    ref = po.fit_lm(c["X"], c["y"])
    for r in range(3):
        assert rel(res[r].coefs, ref["coefs"]) < 1e-10 and rel(res[r].stderr, ref["stderr"]) < 1e-10


def test_external_partials_of_the_wrong_length_are_refused(golden):
    c = golden["logit"]
    X, y = c["X"], c["y"]
    p = X.shape[1]
    good = lambda mode, b, mu0, ybar: po.shard_partials(X, y, "binomial", "logit", mode, b, mu0, ybar)
    for bad in (lambda *a: np.append(good(*a), 1.0), lambda *a: good(*a)[:-1]):
        with pytest.raises(L.IllegalArgumentException):
            D.fit_glm_external(p, lambda: (y.sum(), len(y)), bad)


def test_multi_device_handle_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from sparkglm_amd import Engine
    with pytest.raises(L.SGLMError):
        Engine(devices=[0, 0])


def _collinear_logit(eps, n=20_000, seed=1):
    rng = np.random.default_rng(seed)
    X = np.ones((n, 5))
    X[:, 1] = rng.uniform(-1, 1, n)
    X[:, 2] = X[:, 1] + eps * rng.uniform(-1, 1, n)  # near-duplicate column: cond ~ 6 / eps^2
    X[:, 3] = rng.uniform(-1, 1, n)
    X[:, 4] = X[:, 3] * X[:, 1]
    eta = 0.3 + X[:, 1] - 0.5 * X[:, 3]
    y = (rng.uniform(size=n) < 1 / (1 + np.exp(-eta))).astype(float)
    return np.asfortranarray(X), y


@pytest.mark.parametrize("eps", [1e-2, 1e-4, 1e-5])
def test_ill_conditioned_solve_follows_the_reference_lu(eps):
    """cond(X'WX) from 6e4 to 6e10.  Cholesky and Breeze's LU inverse (utils.scala:103-105) part
    by ~cond * eps (1e-5 relative at 6e10); past the pivot-ratio switch (solve.hpp) the engine
    solves with the reference's LU, so on the same X'WX it reproduces the oracle to rounding."""
    X, y = _collinear_logit(eps)
    n, p = X.shape
    o = po.fit_glm(X, y)
    part = lambda mode, b, mu0, ybar: po.shard_partials(X, y, "binomial", "logit", mode, b, mu0, ybar)
    f = D.fit_glm_external(p, lambda: (y.sum(), n), part)
    w = 1 / (1 + np.exp(-X @ o.coefs))
    cond = np.linalg.cond((X * (w * (1 - w))[:, None]).T @ X)
    assert f.iter == o.iter
    if cond > 1e6:  # LU route: the same algorithm, so 1e-12 on every coefficient (no cond allowance)
        check_fit(f"collinear logit eps {eps:g} (LU route)", f, o, 0.0, tol=1e-12, scalars=False)
    else:  # Cholesky: within 1e-9, or the solve's backward-error scale where that is larger
        check_fit(f"collinear logit eps {eps:g} (Cholesky)", f, o, cond, scalars=False)
    assert rel(f.deviance, o.deviance) < 1e-14


def _adversarial_scalar_fits(golden, allreduce_of):
    """Three ranks whose deviance partials are 1e16, 3 and -1e16 (the Gram is the real shard's):
    the exact sum is 3, a plain all-reduce gives (1e16 + 3) - 1e16 = 4."""
    c = golden["logit"]
    X, y = c["X"], c["y"]
    world, p = 3, X.shape[1]
    devs = [1e16, 3.0, -1e16]
    res, errs = {}, []

    def run(r):
        try:
            lo, hi = D.shard_range(len(y), world, r)
            Xs, ys = np.asfortranarray(X[lo:hi]), y[lo:hi]

            def part(mode, b, mu0, ybar):
                out = po.shard_partials(Xs, ys, "binomial", "logit", mode, b, mu0, ybar)
                out[p * (p + 1) // 2 + p + L.S_DEV] = devs[r]
                return out
            res[r] = D.fit_glm_external(p, lambda: (ys.sum(), len(ys)), part, allreduce=allreduce_of(r))
        except Exception as e:  # pragma: no cover - surfaced below
            errs.append(e)

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    assert not errs, errs
    return res


def test_cross_rank_scalars_are_summed_in_rank_blocks(golden):
    """VERDICT r2 item 3 / SURVEY 8(e) determinism: the per-iteration scalars cross the ranks in
    rank blocks of the all-reduce buffer (every rank's value exact, x + 0 = x) and each rank sums
    them in rank order with compensation -- the in-process communicator's ranks are known to the
    library, so the deviance is the exact 2 * 3; a communicator whose rank the engine does not know
    keeps the plain sum (2 * 4)."""
    comm = D.LocalComm(3)
    res = _adversarial_scalar_fits(golden, comm.rank)
    comm.close()
    for r in range(3):
        assert res[r].deviance == 6.0 and res[r].null_deviance == 6.0 and res[r].iter == 1

    # a Python all-reduce over the same three threads, rank unknown to the engine: plain sums
    bar = threading.Barrier(3)
    bufs = {}

    def plain(r):
        def fn(ptr, count, stream, on_device):
            a = np.ctypeslib.as_array((C.c_double * count).from_address(ptr))
            bufs[r] = a
            bar.wait()
            tot = np.zeros(count)
            for k in range(3):  # rank order, plain
                tot = tot + bufs[k]
            bar.wait()
            a[:] = tot
            bar.wait()
        return fn
    res = _adversarial_scalar_fits(golden, plain)
    assert all(res[r].deviance == 8.0 for r in range(3))


def _chol_solve_unblocked(packed, p):
    """The host solve restated element by element in the order of the unblocked left-looking (jki)
    Cholesky + two column sweeps (solve.cpp before the 4-column panels): every a - b * c is a product
    rounded, then a difference rounded, exactly as the C++ does without FMA contraction."""
    import math
    A = [[0.0] * p for _ in range(p)]  # A[col][row]
    for i in range(p):
        for j in range(i + 1):
            A[j][i] = A[i][j] = float(packed[i * (i + 1) // 2 + j])
    for j in range(p):
        Aj = A[j]
        for k in range(j):
            ljk = A[k][j]
            if ljk == 0.0:
                continue
            Ak = A[k]
            for i in range(j, p):
                Aj[i] = Aj[i] - Ak[i] * ljk
        s = math.sqrt(Aj[j])
        Aj[j] = s
        inv = 1.0 / s
        for i in range(j + 1, p):
            Aj[i] = Aj[i] * inv
    t = [float(v) for v in packed[p * (p + 1) // 2: p * (p + 1) // 2 + p]]
    for j in range(p):
        t[j] = t[j] / A[j][j]
        for i in range(j + 1, p):
            t[i] = t[i] - A[j][i] * t[j]
    for i in range(p - 1, -1, -1):
        t[i] = t[i] / A[i][i]
        for k in range(i):
            t[k] = t[k] - A[k][i] * t[i]
    return np.array(t)


@pytest.mark.parametrize("p", [5, 37, 64])
def test_panel_cholesky_is_bitwise_the_unblocked_factor(p):
    """solve.cpp factors four columns at a time (8-row register blocks, AVX2, no FMA): the LM
    coefficients (LM.scala:225-227, the Cholesky solve of X'X b = X'y) equal, bit for bit, the
    unblocked factorization's restated in Python -- p = 5 / 37 cover a partial last panel and rows
    past the last 8-row block."""
    rng = np.random.default_rng(p)
    X = np.asfortranarray(rng.normal(size=(400, p)))
    y = X @ rng.normal(size=p) + rng.normal(size=400)
    seen = {}

    def part(mode, b, mu0, ybar):
        v = po.shard_partials(X, y, "gaussian", "identity", mode, b, mu0, ybar)
        seen.setdefault(mode, v.copy())
        return v
    f = D.fit_lm_external(p, lambda: (y.sum(), len(y)), part)
    np.testing.assert_array_equal(f.coefs, _chol_solve_unblocked(seen[3], p))
