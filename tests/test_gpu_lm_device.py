"""LM.fit in one device round trip and one pass over X (engine.cpp lm_device; driver.cpp lm_drive):
the LM Gram pass also sums X'1 and y'y (narrow LMX), lm_chol_kernel restates the host Cholesky on the
device (the same operation order, no contraction) and forms LM.scala:160-188's three residual sums
from the Gram pass's sums -- SSE = y'y - 2 b'X'y + b'X'X b, sum (Xb - ybar)^2, sum (y - ybar)^2 --
then one copy back and one synchronisation per fit (BASELINE configs[0] is launch- and latency-
bound).  lm_drive keeps its host solve as the arbiter: the coefficients and inv(X'X) are BITWISE those
of the two-round-trip path (SGLM_LM_DEVICE=0, which runs the reference's residual pass); the
statistics agree with it to rounding (1e-12 here; the oracle bar is 1e-9).  Where the sums cancel
(LM_ONEPASS_MAX_RATIO, e.g. an intercept-only model, whose sum (Xb - ybar)^2 is 0), or the host
leaves Cholesky for the reference's LU inverse (an ill-conditioned X'X), lm_drive reruns the residual
pass at the host's coefficients -- bitwise the host path again (LM.scala:142-237, 241-274)."""
import os

import numpy as np
import pytest

import pyoracle as po
from conftest import rel
from sparkglm_amd import Engine, synth

pytestmark = pytest.mark.gpu


def _engine(device: bool) -> Engine:
    saved = os.environ.get("SGLM_LM_DEVICE")
    os.environ["SGLM_LM_DEVICE"] = "1" if device else "0"
    try:
        return Engine(0)
    finally:
        if saved is None:
            os.environ.pop("SGLM_LM_DEVICE", None)
        else:
            os.environ["SGLM_LM_DEVICE"] = saved


def _fits(load):
    out = {}
    for device in (True, False):
        with _engine(device) as e:
            load(e)
            f = e.fit_lm()
            st = e.stats()
            out[device] = (f, st["lm_device_fits"], st["lm_device_reruns"], st["lm_onepass_fits"])
    return out


def _same(a, b, onepass=False, tol=1e-12):
    """The device fit against the host path's: coefficients and inv(X'X) bitwise; the statistics
    bitwise when the device reran the residual pass, to rounding (`tol`) when they came from the sums."""
    for k in ("coefs", "xtxi"):
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k))
    sa, sb = [a.sse, a.r2, a.fstat, a.sigma, a.nrow], [b.sse, b.r2, b.fstat, b.sigma, b.nrow]
    if onepass:
        assert rel(sa, sb) < tol and rel(a.stderr, b.stderr) < tol, (rel(sa, sb), rel(a.stderr, b.stderr))
    else:
        # (array_equal: an intercept-only model's F statistic is NaN on both paths)
        np.testing.assert_array_equal(sa, sb)
        np.testing.assert_array_equal(a.stderr, b.stderr)


def test_config0_design_bitwise_the_host_path_and_the_oracle():
    n, p = 1_000_000, 20
    res = _fits(lambda e: e.synth(1, 0, n, p, 1))
    (fd, nd, rd, od), (fh, nh, _, _) = res[True], res[False]
    assert nd == 1 and nh == 0 and rd == 0  # the device Cholesky's coefficients were the host's, bitwise
    assert od == 1  # one pass over X: the statistics from the Gram pass's sums
    _same(fd, fh, onepass=True)
    X, y, _, _ = synth.generate(1, 0, n, p, 1)
    r = po.fit_lm(X, y, nthreads=8)
    assert rel(fd.coefs, r["coefs"]) < 1e-9 and rel(fd.stderr, r["stderr"]) < 1e-9
    assert rel([fd.sse, fd.r2, fd.fstat, fd.sigma], [r["sse"], r["r2"], r["fstat"], r["sigma"]]) < 1e-9


@pytest.mark.parametrize("p", [1, 7, 8, 9, 20, 33, 48, 57, 64])
def test_widths_bitwise_the_host_path(p):
    rng = np.random.default_rng(p)
    n = 50_001
    X = np.column_stack([np.ones(n), rng.uniform(-1, 1, (n, p - 1))]) if p > 1 else np.ones((n, 1))
    y = X @ rng.normal(size=p) + rng.uniform(-1, 1, n)
    res = _fits(lambda e: e.set_data(X, y))
    _, nd, rd, od = res[True]
    assert nd == 1
    if p == 1:  # intercept only: sum (Xb - ybar)^2 cancels to rounding -> flagged, the residual pass
        assert od == 0 and rd == 1
    else:  # device coefficients bitwise the host solve's, the statistics from the sums
        assert od == 1 and rd == 0
    _same(res[True][0], res[False][0], onepass=od == 1)


def test_ill_conditioned_falls_back_to_the_host_lu():
    """cond(X'X) ~1e10: the host solver takes the reference's LU inverse (solve.cpp LU_SWITCH_RATIO);
    the device Cholesky flags it and lm_drive reruns the residual pass at the LU coefficients."""
    rng = np.random.default_rng(5)
    n = 20_000
    x1 = rng.uniform(-1, 1, n)
    X = np.column_stack([np.ones(n), x1, x1 + 1e-5 * rng.uniform(-1, 1, n), rng.uniform(-1, 1, (n, 3))])
    y = X @ np.array([1.0, 2.0, -1.0, 0.5, 0.25, -0.75]) + rng.uniform(-1, 1, n)
    res = _fits(lambda e: e.set_data(X, y))
    assert res[True][1] == 1 and res[True][2] == 1  # flagged on the device, rerun at the LU coefficients
    _same(res[True][0], res[False][0])  # the residual pass at the host's coefficients: bitwise
    r = po.fit_lm(X, y)
    assert rel(res[True][0].sse, r["sse"]) < 1e-9


def _fit_or_exc(e):
    try:
        return e.fit_lm()
    except Exception as exc:  # noqa: BLE001
        return type(exc)


@pytest.mark.parametrize("kind", ["zero_column", "duplicate_column"])
def test_rank_deficient_design_takes_the_host_path(kind):
    # a pivot that is not positive makes lm_chol_kernel return NaN coefficients, and
    # lm_drive then never uses the device's residual statistics -- the fit (or its
    # MatrixSingularException) is the two-round-trip path's, bit for bit
    rng = np.random.default_rng(11)
    n = 50_000
    X = np.asfortranarray(np.c_[np.ones(n), rng.uniform(-1, 1, (n, 4))])
    if kind == "zero_column":
        X[:, 3] = 0.0  # X'X has an exactly zero diagonal: the device pivot is 0
    else:
        X[:, 3] = X[:, 1]  # exactly rank deficient
    y = X[:, :3] @ np.array([1.0, 0.5, -0.25]) + rng.uniform(-1, 1, n)
    out = {}
    for device in (True, False):
        with _engine(device) as e:
            e.set_data(X, y)
            out[device] = (_fit_or_exc(e), e.stats())
    fd, fh = out[True][0], out[False][0]
    if isinstance(fd, type):
        assert fd is fh, (fd, fh)
    else:
        assert not isinstance(fh, type)
        _same(fd, fh)
        assert out[True][1]["lm_device_reruns"] == 1  # the host's coefficients, the host's residual pass


@pytest.mark.parametrize("p", [17, 18, 19, 20, 21])
def test_last_column_block_on_4x4_mfma_matches_the_oracle(p):
    """p <= 20 runs the LM Gram (and the gaussian passes) with the second column block's two tiles on
    v_mfma_f64_4x4x4f64 (narrow.hip gram_kstep T4); p = 21 is the first width back on 16x16x4."""
    rng = np.random.default_rng(100 + p)
    n = 200_003
    X = np.column_stack([np.ones(n), rng.uniform(-1, 1, (n, p - 1))])
    y = X @ rng.normal(size=p) + rng.uniform(-1, 1, n)
    with Engine(0) as e:
        e.set_data(X, y)
        f = e.fit_lm()
        g = e.fit_glm("gaussian", "identity")
    r = po.fit_lm(X, y, nthreads=8)
    assert rel(f.coefs, r["coefs"]) < 1e-9 and rel(f.stderr, r["stderr"]) < 1e-9
    assert rel([f.sse, f.r2, f.fstat, f.sigma], [r["sse"], r["r2"], r["fstat"], r["sigma"]]) < 1e-9
    o = po.fit_glm(X, y, "gaussian", "identity", nthreads=8)
    assert g.iter == o.iter
    assert rel(g.coefs, o.coefs) < 1e-9 and rel(g.stderr, o.stderr) < 1e-9
    assert rel([g.deviance, g.null_deviance], [o.deviance, o.null_deviance]) < 1e-9


@pytest.mark.parametrize("shift", [0.0, 30.0, 1e2, 1e4])
def test_onepass_statistics_guard_against_cancellation(shift):
    """y shifted far from 0 (y'y >> SSE, bot): past LM_ONEPASS_MAX_RATIO = 1e4 of max(y'y, b'X'Xb,
    n ybar^2) over min(SSE, top, bot) the sums cancel too far and the statistics come from the residual
    pass (bitwise the host path); below it from the sums, within 1e-12 of the host path.  The oracle
    bar (1e-9) holds either way."""
    rng = np.random.default_rng(21)
    n, p = 100_003, 6
    X = np.column_stack([np.ones(n), rng.uniform(-1, 1, (n, p - 1))])
    y = shift + X @ rng.normal(size=p) + rng.uniform(-1, 1, n)
    res = _fits(lambda e: e.set_data(X, y))
    fd, nd, rd, od = res[True]
    r = po.fit_lm(X, y)
    fit = X @ r["coefs"]
    yb = y.mean()
    big = max(float(y @ y), float(fit @ fit), n * yb * yb)
    small = min(r["sse"], float(np.sum((fit - yb) ** 2)), float(np.sum((y - yb) ** 2)))
    assert abs(np.log10(big / small) - 4.0) > 0.2  # (no case sits on the guard's edge)
    assert od == (1 if big < 1e4 * small else 0), big / small
    # the sums' rounding relative to the statistics grows with big / small (5.5e3 at shift 30)
    _same(fd, res[False][0], onepass=od == 1, tol=max(1e-12, 1e-14 * big / small))
    assert rel([fd.sse, fd.r2, fd.fstat, fd.sigma], [r["sse"], r["r2"], r["fstat"], r["sigma"]]) < 1e-9
