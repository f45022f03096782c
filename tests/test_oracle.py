"""The CPU restatement (oracle/) against everything the reference and independent
implementations pin.  CPU only."""
import json
import os

import numpy as np
import pytest
from scipy import optimize, special

import pyoracle as po
from conftest import GOLDEN, iris_design, rel


def test_iris_r2_matches_reference_known_answer(iris):
    # R/pkg/tests/testthat/test_LM.R:44: "Multiple R-Squared: 3.8443, Adusted R-Squared: 3.9228"
    X, y, _ = iris_design(iris)
    r = po.fit_lm(X, y)
    n, p = X.shape
    adj = 1 - ((1 - r["r2"]) * (n - 1)) / (n - p - 1)
    assert round(r["r2"], 4) == 3.8443
    assert round(adj, 4) == 3.9228


def test_lm_numeric_json_matches_lstsq():
    rows = [json.loads(l) for l in open(os.path.join(GOLDEN, "linear_reg_all_numeric.json"))]
    X = np.array([[r["intercept"]] + [r[f"x{i}"] for i in range(1, 7)] for r in rows])
    y = np.array([r["y"] for r in rows])
    for npart in (1, 4):
        r = po.fit_lm(X, y, npart=npart, nthreads=npart)
        b, *_ = np.linalg.lstsq(X, y, rcond=None)
        assert rel(r["coefs"], b) < 1e-10
        n, p = X.shape
        sig2 = ((y - X @ b) ** 2).sum() / (n - p)
        se = np.sqrt(sig2 * np.diag(np.linalg.inv(X.T @ X)))
        assert rel(r["stderr"], se) < 1e-10
    # SURVEY.md 8c sanity anchor
    assert abs(r["r2"] - 0.353077) < 1e-6 and abs(r["fstat"] - 90.3263) < 1e-4


def test_lm_test_rdd_single_vs_partitioned():
    d = np.loadtxt(os.path.join(GOLDEN, "test_rdd.csv"), delimiter=",", skiprows=1)
    X, y = d[:, :2], d[:, 2]
    a, b = po.fit_lm(X, y, npart=1), po.fit_lm(X, y, npart=4, nthreads=4)
    assert rel(a["coefs"], b["coefs"]) < 1e-12 and rel(a["stderr"], b["stderr"]) < 1e-12
    assert abs(a["r2"] - b["r2"]) < 1e-12


def test_normal_quantile_and_cdf():
    q = np.array([1e-9, 1e-5, 0.01, 0.3, 0.5, 0.77, 0.999, 1 - 1e-9])
    ours = np.array([po.lib().orc_norm_icdf(v) for v in q])
    # Breeze formulation sqrt(2)*erfinv(2q-1): exact up to the cancellation in 2q-1
    assert np.all(np.abs(ours - special.ndtri(q)) <= 1e-15 + 2e-16 / np.maximum(q * (1 - q), 1e-300) * 5)
    x = np.linspace(-6, 6, 25)
    cdf = np.array([po.lib().orc_norm_cdf(v) for v in x])
    assert np.max(np.abs(cdf - special.ndtr(x))) < 2e-16 * 8


def test_lu_inverse_matches_numpy():
    rng = np.random.default_rng(3)
    A = rng.normal(size=(40, 40))
    assert rel(po.lu_inverse(A), np.linalg.inv(A)) < 1e-9
    with pytest.raises(np.linalg.LinAlgError):
        po.lu_inverse(np.zeros((3, 3)))


def _mle(X, y, nll, start=None):
    x0 = np.zeros(X.shape[1]) if start is None else start
    r = optimize.minimize(nll, x0, method="BFGS", options={"gtol": 1e-10, "maxiter": 10000})
    return r.x


def test_glm_binomial_links_match_independent_mle(golden):
    for name, link in (("logit", "logit"), ("probit", "probit"), ("cloglog", "cloglog")):
        c = golden[name]
        X, y = c["X"], c["y"]
        f = po.fit_glm(X, y, "binomial", link)
        if link == "logit":
            p = lambda b: special.expit(X @ b)
        elif link == "probit":
            p = lambda b: special.ndtr(X @ b)
        else:
            p = lambda b: -np.expm1(-np.exp(X @ b))
        nll = lambda b: -np.sum(y * np.log(p(b)) + (1 - y) * np.log1p(-p(b)))
        b = _mle(X, y, nll, start=0.5 * f.coefs)  # independent optimiser from a perturbed start
        assert rel(f.coefs, b) < 1e-4, name
        # IRLS converges to the MLE; the deviance is 2 * nll for 0/1 responses
        assert abs(f.deviance - 2 * nll(f.coefs)) < 1e-8 * f.deviance


def test_glm_poisson_and_gamma_match_independent_mle(golden):
    c = golden["poisson_offset_prior"]
    X, y, off, w = c["X"], c["y"], c["offset"], c["prior"]
    f = po.fit_glm(X, y, "poisson", "log", offset=off, prior=w)
    nll = lambda b: -np.sum(w * (y * (X @ b + off) - np.exp(X @ b + off)))
    assert rel(f.coefs, _mle(X, y, nll)) < 1e-5
    c = golden["gamma"]
    X, y = c["X"], c["y"]
    f = po.fit_glm(X, y, "gamma", "inverse")
    nll = lambda b: np.sum(np.log(1 / (X @ b)) + y * (X @ b)) if np.all(X @ b > 0) else 1e30
    assert rel(f.coefs, _mle(X, y, nll, start=0.8 * f.coefs)) < 1e-4


def test_gaussian_glm_equals_lm_in_two_iterations(golden):
    c = golden["gaussian"]
    f = po.fit_glm(c["X"], c["y"], "gaussian", "identity")
    r = po.fit_lm(c["X"], c["y"])
    assert f.iter == 2 and abs(f.dev_trace[2] - f.dev_trace[1]) <= 4 * np.spacing(f.dev_trace[1])
    assert rel(f.coefs, r["coefs"]) < 1e-12
    n, p = c["X"].shape
    assert rel(f.stderr * np.sqrt(f.deviance / (n - p)), r["stderr"]) < 1e-10


def test_multi_partition_semantics_close_to_single(golden):
    c = golden["logit"]
    a = po.fit_glm(c["X"], c["y"], npart=1)
    b = po.fit_glm(c["X"], c["y"], npart=4, nthreads=4)
    assert a.iter == b.iter and rel(a.coefs, b.coefs) < 1e-12


def test_oracle_reproduces_golden_vectors(golden):
    for name, c in golden.items():
        fam, link, npart = (str(v) for v in c["meta"])
        f = po.fit_glm(c["X"], c["y"], fam, link, m=c.get("m"), offset=c.get("offset"), prior=c.get("prior"),
                       npart=int(npart), nthreads=1)
        s = c["scalars"]
        assert f.iter == int(s[4]), name
        if os.environ.get("SGLM_ORACLE_LIB"):  # another build (sanitizers, -O1): its own summation order
            assert rel(f.coefs, c["coefs"]) < 1e-12 and rel(f.stderr, c["stderr"]) < 1e-12, name
            assert rel([f.deviance, f.null_deviance, f.pearson, f.loglik], s[:4]) < 1e-12, name
            continue
        np.testing.assert_array_equal(f.coefs, c["coefs"], err_msg=name)
        np.testing.assert_array_equal(f.stderr, c["stderr"], err_msg=name)
        np.testing.assert_array_equal(np.array([f.deviance, f.null_deviance, f.pearson, f.loglik]), s[:4])


def test_reference_quirk_mu0_above_m_gives_nan_after_one_iteration(golden):
    c = golden["binomial_m_quirk"]
    assert int(c["scalars"][4]) == 1 and np.isnan(c["scalars"][0])
