"""The C oracle against an INDEPENDENT restatement of the reference (oracle/np_reference.py:
vectorised numpy / scipy written straight from GLM.scala / utils.scala, Breeze inv as LAPACK
dgetrf + dgetri, Breeze Gaussian / Binomial from their published definitions).  The C oracle and
the HIP kernels share one author; this pins the reference-specific semantics a common misreading
would slip past the GPU parity tests:

  * the iteration count (absolute tol on |delta deviance|, deltad starting at 1.0; GLM.scala:281);
  * stdErr from the W of the LAST solve, i.e. the previous iterate's weights (utils.scala:103-105);
  * the null deviance at mu0 = mean(y) (GLM.scala:271, 443), also in fitMultipleBinomial where
    zwCreateBinomial re-derives mu = unlink(link(mean(y))) (GLM.scala:370-371);
  * Pearson with the binomial variance (GLM.scala:95-99);
  * llBinomial's Binomial(m.toInt, mu) with mu as the probability (GLM.scala:140), NaN quirk included.

Bar: identical iteration count; coefficients / stdErr / deviance / null deviance / Pearson /
loglik and the whole deviance trajectory within 1e-12 relative -- for the coefficients and stdErr
max(1e-12, 20 cond(X'WX) eps): two correct summation orders of X'WX part by ~cond * eps in the
solve (gamma/inverse designs here reach cond ~1e4-1e5).  CPU only."""
import numpy as np
import pytest

import np_reference as npr
import pyoracle as po
from conftest import rel
from sparkglm_amd import synth

EPS = np.finfo(float).eps


def _cond(X, y, f, family, link, m=None, off=None, pr=None):
    """cond of the X'WX the last solve inverted (weights at the second-to-last iterate)."""
    n = len(y)
    m = np.ones(n) if m is None else m
    if f.iter < 2:
        return 1.0
    prev = npr.fit_glm(X, y, family, link, m=m, offset=off, prior=pr, max_iter=f.iter - 1)
    mu = npr.unlink(family, link, X @ prev.coefs + (0 if off is None else off), m)
    g = npr.lprime(family, link, mu, m)
    w = (1.0 if pr is None else pr) / (npr.variance(family, mu, m) * g * g)
    return float(np.linalg.cond((X.T * w) @ X))


def _check(X, y, family, link, m=None, off=None, pr=None, npart=1):
    a = npr.fit_glm(X, y, family, link, m=m, offset=off, prior=pr, npart=npart)
    b = po.fit_glm(X, y, family, link, m=m, offset=off, prior=pr, npart=npart, nthreads=1)
    assert a.iter == b.iter
    bar = max(1e-12, 20 * _cond(X, y, b, family, link, m, off, pr) * EPS) if np.isfinite(b.deviance) else 1e-12
    assert rel(a.coefs, b.coefs) < bar and rel(a.stderr, b.stderr) < bar, (rel(a.coefs, b.coefs), bar)
    assert rel([a.deviance, a.null_deviance, a.pearson, a.loglik], [b.deviance, b.null_deviance, b.pearson,
                                                                    b.loglik]) < 1e-12
    assert rel(a.dev_trace, b.dev_trace) < 1e-12
    return a, b


def test_every_golden_case(golden):
    for name, c in golden.items():
        fam, link, npart = (str(v) for v in c["meta"])
        a, _ = _check(c["X"], c["y"], fam, link, c.get("m"), c.get("offset"), c.get("prior"), int(npart))
        # and the committed golden vectors themselves
        s = c["scalars"]
        assert a.iter == int(s[4]), name
        assert rel(a.coefs, c["coefs"]) < 1e-11 and rel([a.deviance, a.null_deviance], s[:2]) < 1e-12, name


SYNTH = [  # (kind, rows, p, family, link): the bench generator at p in {3, 64, 256} and the other links
    (0, 5000, 3, "binomial", "logit"),
    (2, 30000, 64, "poisson", "log"),
    (0, 20000, 256, "binomial", "logit"),
    (0, 30000, 64, "binomial", "probit"),
    (0, 20000, 40, "binomial", "cloglog"),
    (3, 20000, 30, "gamma", "inverse"),
    (1, 20000, 20, "gaussian", "identity"),
]


@pytest.mark.parametrize("npart", [1, 4])
@pytest.mark.parametrize("case", SYNTH, ids=[f"{c[3]}-{c[4]}-p{c[2]}" for c in SYNTH])
def test_synthetic_designs(case, npart):
    kind, n, p, fam, link = case
    X, y, off, pr = synth.generate(kind, 0, n, p, 100 + p)
    _check(X, y, fam, link, off=off, pr=pr, npart=npart)


def test_null_deviance_is_at_mean_y_and_stderr_from_last_solve():
    """The two semantics a restatement most easily gets wrong, spelled out: the null deviance
    is devBinomial at mu0 = mean(y) itself, and stdErr = sqrt(diag(inv(X'W X))) with W from the
    iterate BEFORE the returned coefficients (the solve that produced them)."""
    X, y, _, _ = synth.generate(0, 0, 4000, 6, 7)
    f = po.fit_glm(X, y)
    mu0 = np.full(len(y), y.mean())
    assert rel(f.null_deviance, 2 * np.sum(npr.dev_rows("binomial", y, mu0, np.ones(len(y)), 1.0))) < 1e-12
    prev = npr.fit_glm(X, y, max_iter=f.iter - 1)
    mu = 1 / (1 + np.exp(-(X @ prev.coefs)))
    XtWXi = npr.breeze_inv((X.T * (mu * (1 - mu))) @ X)
    assert rel(f.stderr, np.sqrt(np.diag(XtWXi))) < 1e-12
    # with the weights at the returned coefficients instead, the standard errors move visibly
    mu1 = 1 / (1 + np.exp(-(X @ f.coefs)))
    other = np.sqrt(np.diag(npr.breeze_inv((X.T * (mu1 * (1 - mu1))) @ X)))
    assert rel(other, f.stderr) > 1e-11  # 2e-10 here: far above the 1e-12 agreement above
