"""Parity of the wide-design path (wide.hip: row kernel + panel-pair Gram kernel + rocSOLVER
solve) against the oracle.

The path runs natively for p > 256; SGLM_FORCE_WIDE=1 (read when an engine is created)
routes small designs through it too, so every golden case and the panel-edge shapes are
covered.  Bar as everywhere: coefficients / standard errors / deviance within 1e-9
relative, same iteration count; Gramians norm-wise within 1e-13.  Fits against the oracle go
through conftest.check_fit: each coefficient within 1e-9 or, on an ill-conditioned X'WX, within
the solve's backward-error scale (conftest.coef_bound), with the margin printed."""
import os

import numpy as np
import pytest

import pyoracle as po
from conftest import check_fit, gram_cond, nrel, rel
from sparkglm_amd import Engine, synth

pytestmark = pytest.mark.gpu
TOL = 1e-9


@pytest.fixture(scope="module")
def weng():
    old = os.environ.get("SGLM_FORCE_WIDE")
    os.environ["SGLM_FORCE_WIDE"] = "1"
    try:
        e = Engine(0)
    finally:
        if old is None:
            del os.environ["SGLM_FORCE_WIDE"]
        else:
            os.environ["SGLM_FORCE_WIDE"] = old
    yield e
    e.close()


@pytest.fixture(scope="module")
def eng():
    e = Engine(0)
    yield e
    e.close()


def _logit_pass_check(e, X, y, beta):
    G, xz, s = e.irls_pass(beta)
    eta = X @ beta
    mu = 1 / (1 + np.exp(-eta))
    w = mu * (1 - mu)
    z = eta + (y - mu) / w
    assert nrel(G, (X * w[:, None]).T @ X) < 1e-13
    assert nrel(xz, X.T @ (w * z)) < 1e-13
    dev = np.sum(y * np.log(np.maximum(y, 1) / mu) + (1 - y) * np.log(np.maximum(1 - y, 1) / (1 - mu)))
    assert rel(s[0], dev) < 1e-12
    return G


@pytest.mark.parametrize("p", [1, 2, 17, 64, 127, 128, 129, 200, 256])
def test_forced_wide_gram(weng, p):
    rng = np.random.default_rng(p)
    n = 3000 + 7 * p
    X = rng.uniform(-1, 1, (n, p))
    X[:, 0] = 1.0
    y = (rng.uniform(size=n) < 0.4).astype(float)
    weng.set_data(X, y)
    _logit_pass_check(weng, X, y, rng.normal(size=p) * 0.2)
    st = weng.stats()
    assert st["path"] == 1 and st["wide_panels"] == (p + 127) // 128


@pytest.mark.parametrize("p", [257, 300, 384, 520, 1030])
def test_native_wide_gram(eng, p):
    rng = np.random.default_rng(p)
    n = 3000 + 7 * p
    X = rng.uniform(-1, 1, (n, p)) / np.sqrt(p)
    X[:, 0] = 1.0
    y = (rng.uniform(size=n) < 0.4).astype(float)
    eng.set_data(X, y)
    _logit_pass_check(eng, X, y, rng.normal(size=p) * 0.5)
    assert eng.stats()["path"] == 1


def test_forced_wide_golden_cases(weng, golden):
    for name, c in golden.items():
        fam, link, npart = (str(v) for v in c["meta"])
        weng.set_data(c["X"], c["y"], c.get("m"), c.get("offset"), c.get("prior"))
        f = weng.fit_glm(fam, link, init="multiple" if npart != "1" else "single")
        s = c["scalars"]
        assert f.iter == int(s[4]), name
        if np.isnan(s[0]):
            assert np.isnan(f.deviance), name
            continue
        assert rel(f.coefs, c["coefs"]) < TOL, name
        assert rel(f.stderr, c["stderr"]) < TOL, name
        assert rel([f.deviance, f.null_deviance, f.pearson, f.loglik], s[:4]) < TOL, name
        assert rel(f.dev_trace, c["trace"]) < TOL, name


def test_forced_wide_edge_shapes(weng):
    rng = np.random.default_rng(11)
    for n, p in ((1, 1), (5, 1), (31, 2), (32, 3), (33, 3), (64, 16), (65, 130)):
        X = rng.uniform(-1, 1, (n, p))
        X[:, 0] = 1.0
        y = rng.normal(size=n) + 3
        weng.set_data(X, y)
        G, xz, s = weng.irls_pass(np.zeros(p), family="gaussian", link="identity")
        assert nrel(G, X.T @ X) < 1e-13 and nrel(xz, X.T @ y) < 1e-13
        if n > p:
            f = weng.fit_lm()
            r = po.fit_lm(X, y)
            assert rel(f.coefs, r["coefs"]) < TOL and rel(f.stderr, r["stderr"]) < TOL
            assert rel(f.xtxi, r["xtxi"]) < 1e-8


def _gamma_data(n, p, seed):
    rng = np.random.default_rng(seed)
    X = rng.uniform(0.5, 1.5, (n, p)) / p
    X[:, 0] = 1.0
    beta = np.full(p, 0.5)
    mu = 1.0 / (X @ beta)
    y = rng.gamma(5.0, mu / 5.0)
    return X, y


@pytest.mark.parametrize("case", ["logit300", "probit264", "poisson300", "gamma260", "cloglog520"])
def test_native_wide_fits_match_oracle(eng, case):
    kw = {}
    if case == "logit300":
        X, y, _, _ = synth.generate(0, 0, 15000, 300, 31)
        fam, link = "binomial", "logit"
    elif case == "probit264":
        X, y, _, _ = synth.generate(0, 0, 12000, 264, 32)
        fam, link = "binomial", "probit"
    elif case == "poisson300":
        X, y, off, pr = synth.generate(2, 0, 15000, 300, 33)
        fam, link = "poisson", "log"
        kw = dict(offset=off, prior=pr)
    elif case == "gamma260":
        X, y = _gamma_data(12000, 260, 34)
        fam, link = "gamma", "inverse"
    else:
        X, y, _, _ = synth.generate(0, 0, 20000, 520, 35)
        y = (synth.unif(np.arange(20000, dtype=np.uint64) + np.uint64(91)) < 0.3).astype(float)
        fam, link = "binomial", "cloglog"
    eng.set_data(X, y, offset=kw.get("offset"), prior=kw.get("prior"))
    f = eng.fit_glm(fam, link)
    o = po.fit_glm(X, y, fam, link, nthreads=8, **kw)
    check_fit(case, f, o, gram_cond(eng, f.coefs, fam, link))


def test_native_wide_lm(eng):
    X, y, _, _ = synth.generate(1, 0, 20000, 300, 36)
    eng.set_data(X, y)
    f = eng.fit_lm()
    r = po.fit_lm(X, y, nthreads=8)
    check_fit("lm300", f, r, gram_cond(eng, f.coefs, "gaussian", "identity"), scalars=False)
    assert rel([f.sse, f.r2, f.fstat, f.sigma], [r["sse"], r["r2"], r["fstat"], r["sigma"]]) < TOL


def test_wide_large_properties(eng):
    """1M x 512 resident logit fit: a 20k-row prefix against the oracle, then at full size the
    score equation at the MLE, monotone deviance and bitwise run-to-run determinism."""
    p = 512
    eng.synth(0, 0, 20_000, p, 5)
    X, y, _, _, _ = eng.get_data()
    f = eng.fit_glm()
    o = po.fit_glm(X, y, nthreads=8)
    check_fit("logit512 20k prefix", f, o, gram_cond(eng, f.coefs))
    del X, y
    eng.synth(0, 0, 1_000_000, p, 5)
    f = eng.fit_glm()
    assert np.all(np.diff(f.dev_trace[: f.iter + 1]) <= 1e-6)
    G, xz, _ = eng.irls_pass(f.coefs)
    assert np.max(np.abs(xz - G @ f.coefs)) < 1e-6 * np.max(np.abs(xz))
    g = eng.fit_glm()
    np.testing.assert_array_equal(f.coefs, g.coefs)
    np.testing.assert_array_equal(f.stderr, g.stderr)


@pytest.mark.parametrize("p", [64, 1100])
def test_gamma_synth_design_device_generated(eng, p):
    """BASELINE configs[3]'s design (synth kind 3: positive X, gamma/inverse) generated in HBM by
    the device generator; the oracle fits the bit-identical host copy."""
    n = 9000
    eng.synth(3, 1000, n, p, 4)
    X, y, _, _ = synth.generate(3, 1000, n, p, 4)
    f = eng.fit_glm("gamma", "inverse")
    o = po.fit_glm(X, y, "gamma", "inverse", nthreads=8)
    check_fit(f"gamma synth p{p}", f, o, gram_cond(eng, f.coefs, "gamma", "inverse"))


@pytest.mark.parametrize("kind,p,fam,link", [(0, 300, "binomial", "logit"), (2, 290, "poisson", "log"),
                                             (3, 520, "gamma", "inverse"), (0, 40, "binomial", "logit")])
def test_procedural_shard_is_bitwise_the_resident_fit(eng, kind, p, fam, link):
    """sglm_synth_procedural (X regenerated in the kernels, never stored) gives bit-for-bit the
    fit of the resident image of the same generator, and both match the oracle."""
    n, row0 = 7000, 12345
    eng.synth(kind, row0, n, p, 8)
    res = eng.fit_glm(fam, link)
    res_pred = eng.predict(res.coefs)
    eng.synth(kind, row0, n, p, 8, procedural=True)
    st = eng.stats()
    assert st["path"] == 1  # procedural shards run the wide kernels at any p
    pro = eng.fit_glm(fam, link)
    if p > 256:  # both run the wide kernels: bit-for-bit
        np.testing.assert_array_equal(pro.coefs, res.coefs)
        np.testing.assert_array_equal(pro.stderr, res.stderr)
        assert (pro.deviance, pro.pearson, pro.loglik, pro.iter) == (res.deviance, res.pearson, res.loglik, res.iter)
        np.testing.assert_array_equal(eng.predict(pro.coefs), res_pred)
    else:  # resident p <= 256 runs the fused/narrow pass: another summation order
        assert pro.iter == res.iter and rel(pro.coefs, res.coefs) < 1e-12 and rel(pro.stderr, res.stderr) < 1e-12
    X, y, off, pr = synth.generate(kind, row0, n, p, 8)
    kw = dict(offset=off, prior=pr) if kind == 2 else {}
    o = po.fit_glm(X, y, fam, link, nthreads=8, **kw)
    check_fit(f"procedural kind{kind} p{p}", pro, o, gram_cond(eng, pro.coefs, fam, link))


def test_procedural_lm_and_get_data(eng):
    eng.synth(1, 0, 6000, 300, 9, procedural=True)
    f = eng.fit_lm()
    X, y, _, _ = synth.generate(1, 0, 6000, 300, 9)
    r = po.fit_lm(X, y, nthreads=8)
    check_fit("procedural lm300", f, r, gram_cond(eng, f.coefs, "gaussian", "identity"), scalars=False)
    with pytest.raises(Exception):
        eng.get_data()


def _engine_env(**env) -> Engine:
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return Engine(0)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("kind,p,fam,link", [(0, 300, "binomial", "logit"), (3, 520, "gamma", "inverse")])
def test_wide_solve_lu_and_cholesky(kind, p, fam, link):
    """The wide path's device solves: Cholesky (default) and, with SGLM_WIDE_SOLVE=lu, the
    reference's own algorithm -- LU + explicit inverse (Breeze inv = dgetrf + dgetri,
    utils.scala:103-105) by rocSOLVER, coefs = inv * X'Wz summed in the reference's order -- both
    against the oracle's unblocked LU; sglm_stats.solve_path says which ran.  Well-conditioned
    logit: everything elementwise at 1e-9.  Gamma/inverse at p = 520 (cond ~1e7): blocked LU and
    the unblocked restatement part by ~1e-7 on the smallest coefficient (Cholesky ~1e-9, the
    conditioning floor of DESIGN.md section 3), so coefficients norm-wise at 1e-9 and each within
    the solve's backward-error scale (conftest.coef_bound)."""
    n = 20_000
    X, y, _, _ = synth.generate(kind, 0, n, p, 17)
    o = po.fit_glm(X, y, fam, link, nthreads=8)
    for mode, want in (("lu", "device-lu"), ("chol", "device-cholesky"), ("", "device-cholesky")):
        e = _engine_env(SGLM_WIDE_SOLVE=mode)
        try:
            e.synth(kind, 0, n, p, 17)
            f = e.fit_glm(fam, link)
            st = e.stats()
            cond = gram_cond(e, f.coefs, fam, link)
        finally:
            e.close()
        assert st["path"] == 1 and st["solve_path_name"] == want, st["solve_path_name"]
        assert nrel(f.coefs, o.coefs) < TOL
        check_fit(f"{fam} p{p} {want}", f, o, cond)


def test_wide_singular_gram_raises_matrix_singular(weng):
    """An exactly singular X'WX (a duplicated column) on the device LU route -> Breeze's
    MatrixSingularException, as inv() throws it (utils.scala:103)."""
    from sparkglm_amd import _lib as L
    X, y, _, _ = synth.generate(1, 0, 5000, 6, 3)
    X = np.column_stack([X, X[:, 2]])
    weng.set_data(X, y)
    with pytest.raises(L.MatrixSingularException):
        weng.fit_lm()


@pytest.mark.parametrize("kind,p,fam,link", [(0, 300, "binomial", "logit"), (3, 520, "gamma", "inverse")])
def test_procedural_in_kernel_generation_is_bitwise_the_chunked_fit(kind, p, fam, link):
    """SGLM_PROC_CHUNKS=0 selects the procedural path's fallback for too little free HBM: the Gram
    kernels regenerate every X octet they stage (wide_gram_kernel<..., PROC = true>) instead of
    reading a generated chunk -- the same values in the same order, so the same fit bit for bit."""
    n, row0 = 5000, 4321
    with Engine(0) as e:
        e.synth(kind, row0, n, p, 8, procedural=True)
        assert e.stats()["proc_chunks"] >= 1
        a = e.fit_glm(fam, link)
    with _engine_env(SGLM_PROC_CHUNKS="0") as e:
        e.synth(kind, row0, n, p, 8, procedural=True)
        assert e.stats()["proc_chunks"] == 0
        b = e.fit_glm(fam, link)
    np.testing.assert_array_equal(a.coefs, b.coefs)
    np.testing.assert_array_equal(a.stderr, b.stderr)
    assert (a.deviance, a.pearson, a.loglik, a.iter) == (b.deviance, b.pearson, b.loglik, b.iter)
