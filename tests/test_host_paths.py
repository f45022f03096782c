"""Host-side paths of the C-ABI library that need no GPU: the in-process communicator (N host
threads, one fit each -- a JVM driver's thread pool), the external backend's wire-format check,
the multi-device handle's refusal without a device, and the solve on ill-conditioned designs.
Partials come from the oracle (the checker)."""
import threading

import numpy as np
import pytest

import pyoracle as po
from conftest import rel
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
    tol = 1e-12 if cond > 1e6 else 1e-9  # LU route: the same algorithm; Cholesky: within cond * eps
    assert rel(f.coefs, o.coefs) < tol and rel(f.stderr, o.stderr) < tol, cond
    assert rel(f.deviance, o.deviance) < 1e-14
