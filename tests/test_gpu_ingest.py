"""The ingest boundary, scoring and the single-process multi-device handle on the GPU:

  * sglm_reserve + sglm_set_rows (partition-wise blocks, out of order, through pinned staging)
    give bit-for-bit the fit of one sglm_set_data (utils.scala:36-49's per-partition matrices);
  * sglm_predict_new scores new rows without evicting the resident training design
    (LM.scala:29-61), GLM response-scale prediction = unlink(X beta + offset);
  * sglm_create_multi: one handle over several devices; a device listed twice
    rehearses the sharding on one GPU with host sums, a single device runs the RCCL group path;
  * set_data_device round-trips torch tensors and refuses ones it would misread."""
import numpy as np
import pytest

import pyoracle as po
from conftest import nrel, rel
from sparkglm_amd import Engine, synth
from sparkglm_amd import _lib as L

pytestmark = pytest.mark.gpu
TOL = 1e-9


@pytest.fixture(scope="module")
def eng():
    e = Engine(0)
    yield e
    e.close()


def test_blockwise_upload_is_bitwise_one_upload(eng):
    n, p = 50_003, 40
    X, y, off, pr = synth.generate(2, 0, n, p, 21)
    eng.set_data(X, y, offset=off, prior=pr)
    a = eng.fit_glm("poisson", "log")
    st = eng.stats()
    assert st["load_bytes"] == 8 * n * (p + 3) and st["load_ms"] > 0
    eng.reserve(n, p, offset=True, prior=True)
    cuts = [0, 7, 20_000, 20_001, 41_000, n]
    for k in (3, 0, 4, 2, 1):  # arbitrary order, ragged blocks
        lo, hi = cuts[k], cuts[k + 1]
        eng.set_rows(lo, X[lo:hi], y[lo:hi], offset=off[lo:hi], prior=pr[lo:hi])
    b = eng.fit_glm("poisson", "log")
    np.testing.assert_array_equal(a.coefs, b.coefs)
    np.testing.assert_array_equal(a.stderr, b.stderr)
    assert (a.deviance, a.pearson, a.loglik, a.iter) == (b.deviance, b.pearson, b.loglik, b.iter)
    Xb, yb, _, ob, pb = eng.get_data()
    np.testing.assert_array_equal(Xb, X)
    np.testing.assert_array_equal(ob, off)


def test_incomplete_or_mismatched_upload_is_refused(eng):
    n, p = 1000, 5
    X, y, _, _ = synth.generate(0, 0, n, p, 3)
    eng.reserve(n, p)
    eng.set_rows(0, X[:600], y[:600])
    with pytest.raises(L.IllegalArgumentException, match="never written"):
        eng.fit_glm()
    with pytest.raises(L.IllegalArgumentException):
        eng.set_rows(900, X[:200], y[:200])          # past the reserved rows
    with pytest.raises(L.IllegalArgumentException):
        eng.set_rows(600, X[600:], y[600:], m=np.ones(400))  # m was not reserved
    eng.set_rows(600, X[600:], y[600:])
    f = eng.fit_glm()
    o = po.fit_glm(X, y)
    assert f.iter == o.iter and rel(f.coefs, o.coefs) < TOL


def test_overlapping_blocks_are_refused(eng):
    """a repeated or overlapping block must not count its rows twice -- two
    set_rows(0, n/2) calls would otherwise pass the coverage check with the second half never
    written (zero X, y) and the fit would silently run over it."""
    n, p = 1000, 5
    X, y, _, _ = synth.generate(0, 0, n, p, 3)
    eng.reserve(n, p)
    eng.set_rows(0, X[:500], y[:500])
    with pytest.raises(L.IllegalArgumentException, match="overlap"):
        eng.set_rows(0, X[:500], y[:500])             # the same block again
    with pytest.raises(L.IllegalArgumentException, match="overlap"):
        eng.set_rows(499, X[499:700], y[499:700])     # straddles the written block's end
    eng.set_rows(700, X[700:], y[700:])
    with pytest.raises(L.IllegalArgumentException, match="overlap"):
        eng.set_rows(600, X[600:701], y[600:701])     # straddles the next block's start
    with pytest.raises(L.IllegalArgumentException, match="never written"):
        eng.fit_glm()
    eng.set_rows(500, X[500:700], y[500:700])         # the exact gap
    f = eng.fit_glm()
    o = po.fit_glm(X, y)
    assert f.iter == o.iter and rel(f.coefs, o.coefs) < TOL


def test_predict_new_keeps_the_training_design_resident(eng):
    X, y, off, pr = synth.generate(2, 0, 30_000, 12, 5)
    eng.set_data(X, y, offset=off, prior=pr)
    f = eng.fit_glm("poisson", "log")
    Xn, _, offn, _ = synth.generate(2, 10**6, 7_777, 12, 5)
    eta = eng.predict_new(Xn, f.coefs, "poisson", "log", "link", offset=offn)
    assert rel(eta, Xn @ f.coefs + offn) < 1e-13
    mu = eng.predict_new(Xn, f.coefs, "poisson", "log", "response", offset=offn)
    assert rel(mu, np.exp(Xn @ f.coefs + offn)) < 1e-13
    g = eng.fit_glm("poisson", "log")  # the shard was not evicted
    np.testing.assert_array_equal(f.coefs, g.coefs)
    fitted = eng.predict_glm(f.coefs, "poisson", "log", "response")
    assert rel(fitted, np.exp(X @ f.coefs + off)) < 1e-13


@pytest.mark.parametrize("link", ["logit", "probit", "cloglog"])
def test_binomial_response_prediction(eng, link):
    from scipy.special import ndtr
    X, y, _, _ = synth.generate(0, 0, 20_000, 9, 6)
    eng.set_data(X, y)
    beta = np.linspace(-0.5, 0.5, 9)
    eta = X @ beta
    mu = {"logit": 1 / (1 + np.exp(-eta)), "probit": ndtr(eta), "cloglog": 1 - np.exp(-np.exp(eta))}[link]
    assert rel(eng.predict_glm(beta, "binomial", link, "response"), mu) < 1e-12
    m = 1.0 + np.arange(20_000) % 4
    assert rel(eng.predict_new(X, beta, "binomial", link, "response", m=m), m * mu) < 1e-12
    gam = eng.predict_new(np.abs(X) + 0.1, np.full(9, 0.3), "gamma", "inverse", "response")
    assert rel(gam, 1.0 / ((np.abs(X) + 0.1) @ np.full(9, 0.3))) < 1e-13


def test_api_predict_mirrors():
    from sparkglm_amd.frame import Frame
    from sparkglm_amd.glm import GLM
    from sparkglm_amd.lm import LM
    X, y, _, _ = synth.generate(0, 0, 5_000, 4, 9)
    cols = {f"x{j}": X[:, j] for j in range(4)}
    x = Frame(cols, 1)
    model = GLM.fit(Frame({"y": y}, 1), x, "binomial", "logit")
    pr = model.predict(x, type="response")
    assert rel(pr["value"], 1 / (1 + np.exp(-(X @ np.ravel(model.coefs))))) < 1e-12
    Xl, yl, _, _ = synth.generate(1, 0, 5_000, 4, 9)
    lm = LM.fit(Frame({f"x{j}": Xl[:, j] for j in range(4)}, 1), Frame({"y": yl}, 1))
    out = lm.predict(Frame({f"x{j}": Xl[:, j] for j in range(4)}, 1))
    assert rel(out["value"], Xl @ np.ravel(lm.coefs)) < 1e-13
    with pytest.raises(L.IllegalArgumentException):  # the reference multiplies newData's whole matrix
        lm.predict(Frame({**{f"x{j}": Xl[:, j] for j in range(4)}, "extra": yl}, 1))


@pytest.mark.parametrize("devs", [[0, 0], [0, 0, 0], [0]])
def test_multi_device_handle_matches_partitioned_oracle(devs):
    """sglm_create_multi: shards per listed device.  [0, 0] / [0, 0, 0] share the one GPU (host
    sums in device order), [0] runs the ncclCommInitAll + group all-reduce path."""
    n, p = 90_001, 48
    X, y, off, pr = synth.generate(2, 0, n, p, 5)
    with Engine(devices=devs) as g:
        g.set_data(X, y, offset=off, prior=pr)
        f = g.fit_glm("poisson", "log", init="multiple")
        st = g.stats()
        assert st["ndev"] == len(devs) and st["n_local"] == n and st["rccl_group"] == (1 if devs == [0] else 0)
        o = po.fit_glm(X, y, "poisson", "log", offset=off, prior=pr, npart=len(devs), nthreads=8)
        assert f.iter == o.iter and f.npart == len(devs) and f.nrow == n
        assert rel(f.coefs, o.coefs) < TOL and rel(f.stderr, o.stderr) < TOL
        assert rel([f.deviance, f.null_deviance, f.pearson, f.loglik],
                   [o.deviance, o.null_deviance, o.pearson, o.loglik]) < TOL
        assert nrel(g.predict(f.coefs, add_offset=True), X @ f.coefs + off) < 1e-14
        Xg, yg, _, og, _ = g.get_data()
        np.testing.assert_array_equal(Xg, X)
        # generated shards and the LM path through the same handle
        g.synth(1, 0, 60_000, 20, 1)
        lm = g.fit_lm()
        Xs, ys, _, _ = synth.generate(1, 0, 60_000, 20, 1)
        r = po.fit_lm(Xs, ys)
        assert rel(lm.coefs, r["coefs"]) < TOL and rel(lm.stderr, r["stderr"]) < TOL and lm.npart == len(devs)
        # blockwise ingest across the shard boundaries
        g.reserve(n, p, offset=True, prior=True)
        for lo in range(0, n, 25_000):
            hi = min(n, lo + 25_000)
            g.set_rows(lo, X[lo:hi], y[lo:hi], offset=off[lo:hi], prior=pr[lo:hi])
        h = g.fit_glm("poisson", "log", init="multiple")
        np.testing.assert_array_equal(h.coefs, f.coefs)


def test_multi_device_wide_path():
    X, y, _, _ = synth.generate(0, 0, 9_000, 300, 13)
    with Engine(devices=[0, 0]) as g:
        g.set_data(X, y)
        f = g.fit_glm()
        assert g.stats()["path"] == 1
    o = po.fit_glm(X, y, npart=2, nthreads=8)
    assert f.iter == o.iter and rel(f.coefs, o.coefs) < TOL and rel(f.stderr, o.stderr) < TOL


def test_set_data_device_round_trip_and_validation(eng):
    import torch
    X, y, off, pr = synth.generate(2, 0, 4_000, 10, 7)
    dev = torch.device("cuda", 0)
    tX = torch.from_numpy(X).to(dev).t().contiguous().t()
    ty, toff, tpr = (torch.from_numpy(v).to(dev) for v in (y, off, pr))
    eng.set_data_device(tX, ty, offset=toff, prior=tpr)
    Xb, yb, _, ob, pb = eng.get_data()
    np.testing.assert_array_equal(Xb, X)
    np.testing.assert_array_equal(yb, y)
    np.testing.assert_array_equal(pb, pr)
    with pytest.raises(L.IllegalArgumentException):
        eng.set_data_device(tX.float(), ty)                      # float32
    with pytest.raises(L.IllegalArgumentException):
        eng.set_data_device(tX.contiguous(), ty)                 # row-major
    with pytest.raises(L.IllegalArgumentException):
        eng.set_data_device(tX, torch.from_numpy(np.repeat(y, 2)).to(dev)[::2])  # strided view
    with pytest.raises(L.IllegalArgumentException):
        eng.set_data_device(tX, ty.cpu())                        # host tensor


@pytest.mark.parametrize("eps", [1e-4, 1e-5])
def test_ill_conditioned_design_on_gpu(eng, eps):
    """cond(X'WX) ~ 6e8 / 6e10: the engine's Gram differs from the oracle's by summation-order
    rounding (~1e-16 relative), which any solve amplifies by cond -- the bar here is
    max(1e-9, 50 cond eps), with the solve itself on the reference's LU (solve.hpp switch)."""
    rng = np.random.default_rng(1)
    n = 40_000
    X = np.ones((n, 5))
    X[:, 1] = rng.uniform(-1, 1, n)
    X[:, 2] = X[:, 1] + eps * rng.uniform(-1, 1, n)
    X[:, 3] = rng.uniform(-1, 1, n)
    X[:, 4] = X[:, 3] * X[:, 1]
    y = (rng.uniform(size=n) < 1 / (1 + np.exp(-(0.3 + X[:, 1] - 0.5 * X[:, 3])))).astype(float)
    eng.set_data(X, y)
    f = eng.fit_glm()
    o = po.fit_glm(X, y)
    w = 1 / (1 + np.exp(-X @ o.coefs))
    cond = np.linalg.cond((X * (w * (1 - w))[:, None]).T @ X)
    tol = max(1e-9, 50 * cond * 2.2e-16)
    print(f"\ncond {cond:.2e}: coefs {rel(f.coefs, o.coefs):.2e} stderr {rel(f.stderr, o.stderr):.2e} (bar {tol:.1e})")
    assert f.iter == o.iter
    assert rel(f.coefs, o.coefs) < tol and rel(f.stderr, o.stderr) < tol
    assert rel(f.deviance, o.deviance) < TOL
