"""Bounded waits on the all-reduce (the treeReduce seam, utils.scala:110-126).

A rank whose peer died must fail with SGLM_ECOMM naming itself and what it waited for -- not hang
until an outside time limit.  These run on the CPU through the external-backend fits, which use the
same caller-callback runner (a communicator thread waited on with SGLM_COMM_TIMEOUT_S) as an engine
handle's sglm_set_comm; the device paths (RCCL, a gloo group over device buffers) are in
tests/test_gpu_dist.py."""
import os
import sys
import threading
import time

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "oracle"))


def _case():
    rng = np.random.default_rng(5)
    X = np.asfortranarray(np.c_[np.ones(200), rng.uniform(-1, 1, (200, 3))])
    y = (rng.uniform(size=200) < 0.4).astype(float)
    return X, y


def _backend(X, y):
    import pyoracle as po
    sums = lambda: (y.sum(), len(y))
    part = lambda mode, b, mu0, ybar: po.shard_partials(X, y, "binomial", "logit", mode, b, mu0, ybar)
    return sums, part


def test_caller_allreduce_that_never_returns_fails_within_the_deadline(monkeypatch):
    from sparkglm_amd import distributed as D
    from sparkglm_amd._lib import CommError
    monkeypatch.setenv("SGLM_COMM_TIMEOUT_S", "1")
    X, y = _case()
    sums, part = _backend(X, y)
    release = threading.Event()
    calls = []

    def stuck(ptr, count, stream, on_device):  # a peer that never joins: the collective never returns
        calls.append(threading.get_ident())
        release.wait(60)
        raise RuntimeError("released")

    t0 = time.perf_counter()
    with pytest.raises(CommError) as ei:
        D.fit_glm_external(X.shape[1], sums, part, allreduce=stuck)
    dt = time.perf_counter() - t0
    release.set()
    assert 0.9 < dt < 20.0
    msg = str(ei.value)
    assert "did not return within SGLM_COMM_TIMEOUT_S" in msg and "1.0" in msg
    # the callback ran on the communicator thread, not on the caller's
    assert calls and calls[0] != threading.get_ident()


def test_caller_allreduce_runs_normally_under_the_deadline(monkeypatch):
    # an identity all-reduce (one rank) through the runner: the fit equals the one without a communicator
    from sparkglm_amd import distributed as D
    monkeypatch.setenv("SGLM_COMM_TIMEOUT_S", "30")
    X, y = _case()
    sums, part = _backend(X, y)
    seen = []
    a = D.fit_glm_external(X.shape[1], sums, part, allreduce=lambda p, c, s, d: seen.append(c))
    b = D.fit_glm_external(X.shape[1], sums, part, allreduce=None)
    assert seen and a.iter == b.iter
    assert np.array_equal(a.coefs, b.coefs) and a.deviance == b.deviance


def test_failing_callback_is_reported_with_the_rank(monkeypatch):
    from sparkglm_amd import distributed as D
    from sparkglm_amd._lib import CommError
    monkeypatch.setenv("SGLM_COMM_TIMEOUT_S", "30")
    X, y = _case()
    sums, part = _backend(X, y)

    def bad(ptr, count, stream, on_device):
        raise RuntimeError("peer reset")

    with pytest.raises(CommError, match="caller all-reduce failed"):
        D.fit_glm_external(X.shape[1], sums, part, allreduce=bad)


def test_in_process_communicator_with_a_missing_rank_fails_within_the_deadline(monkeypatch):
    # two-rank in-process communicator, only rank 0 fits: its all-reduce gives up at the deadline
    from sparkglm_amd import distributed as D
    from sparkglm_amd._lib import CommError
    monkeypatch.setenv("SGLM_COMM_TIMEOUT_S", "1")
    X, y = _case()
    sums, part = _backend(X, y)
    comm = D.LocalComm(2)
    try:
        t0 = time.perf_counter()
        with pytest.raises(CommError, match="in-process all-reduce failed on rank 0"):
            D.fit_glm_external(X.shape[1], sums, part, allreduce=comm.rank(0))
        assert 0.9 < time.perf_counter() - t0 < 20.0
    finally:
        comm.close()


def test_unbounded_when_the_timeout_is_zero(monkeypatch):
    # SGLM_COMM_TIMEOUT_S=0: the callback runs inline on the caller's thread (no deadline)
    from sparkglm_amd import distributed as D
    monkeypatch.setenv("SGLM_COMM_TIMEOUT_S", "0")
    X, y = _case()
    sums, part = _backend(X, y)
    tid = []
    D.fit_glm_external(X.shape[1], sums, part, allreduce=lambda p, c, s, d: tid.append(threading.get_ident()))
    assert tid and set(tid) == {threading.get_ident()}
