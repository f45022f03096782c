import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))  # the checker (tests only)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP engine)")


@pytest.fixture(scope="session")
def golden():
    z = np.load(os.path.join(GOLDEN, "glm_golden.npz"), allow_pickle=False)
    cases = {}
    for key in z.files:
        name, field = key.split("/")
        cases.setdefault(name, {})[field] = z[key]
    return cases


@pytest.fixture(scope="session")
def iris():
    import csv
    with open(os.path.join(GOLDEN, "iris.csv")) as f:
        rows = list(csv.DictReader(f))
    cols = {k: np.array([float(r[k]) for r in rows]) for k in rows[0] if k != "Species"}
    cols["Species"] = np.array([r["Species"] for r in rows], dtype=object)
    return cols


def iris_design(iris):
    """Sepal_Width ~ Petal_Length + Petal_Width + Species (test_LM.R:10, 39-44): the R
    modelMatrix drops the first level and adds no intercept."""
    sp = iris["Species"]
    X = np.column_stack([iris["Petal_Length"], iris["Petal_Width"], (sp == "versicolor").astype(float),
                         (sp == "virginica").astype(float)])
    return X, iris["Sepal_Width"], ["Petal_Length", "Petal_Width", "Species_versicolor", "Species_virginica"]


def rel(a, b):
    """Max relative difference; positions that are NaN in both (the reference's own NaN
    quirks, e.g. llBinomial with m > 1) count as equal."""
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    if not a.size:
        return 0.0
    both = np.isnan(a) & np.isnan(b)
    d = np.where(both, 0.0, np.abs(a - b) / np.maximum(np.abs(b), 1e-300))
    return float(np.max(np.where(np.isnan(d), np.inf, d)))


def nrel(a, b):
    """Norm-wise relative difference max|a-b| / max|b| (for sums with cancellation)."""
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / np.max(np.abs(b)))


# Per-coefficient bar for ill-conditioned solves (gamma designs): the solve's backward-error scale
# cond * eps * max|b| / |b_i| times K = 20, the spread the reference's own algorithm shows between two
# correct implementations of it on configs[3]'s X'WX (tests/golden/gram_split_p2048.json: LAPACK
# dgetrf + dgetri against the oracle's unblocked restatement reaches K = 17.6).
K_BOUND = 20.0


def cond_ok(b, r, cond, tol=1e-9, k=K_BOUND):
    b, r = np.asarray(b, dtype=np.float64), np.asarray(r, dtype=np.float64)
    bound = np.maximum(tol, k * cond * np.finfo(float).eps * np.max(np.abs(r)) / np.abs(r))
    return bool(np.all(np.abs(b - r) / np.abs(r) <= bound))


def coef_bound(r, cond, tol=1e-9, k=K_BOUND):
    """Per-coefficient relative bar: `tol`, or on an ill-conditioned solve the backward-error scale
    k * cond * eps * max|b| / |b_i| where that is larger (one bar for every fit,
    whichever path; a well-conditioned design keeps the fixed 1e-9 on every coefficient)."""
    r = np.abs(np.asarray(r, dtype=np.float64))
    return np.maximum(tol, k * cond * np.finfo(float).eps * np.max(r) / np.maximum(r, 1e-300))


def gram_cond(eng, coefs, family="binomial", link="logit"):
    """cond(X'WX) at the fitted coefficients, from one engine pass (the matrix the solve saw)."""
    G, _, _ = eng.irls_pass(np.asarray(coefs, dtype=np.float64), family=family, link=link)
    return float(np.linalg.cond(G))


def check_fit(label, f, o, cond, tol=1e-9, scalars=True):
    """The parity bar of one fit against the oracle's, with its MARGIN printed (bar / error, the
    smallest over the outputs; >= 1 passes): coefficients each within coef_bound, standard errors
    and the deviance-family scalars elementwise within `tol`, the same iteration count.  `o` is an
    oracle fit (attributes) or a dict with coefs / stderr / deviance ... keys."""
    get = (lambda k: o[k]) if isinstance(o, dict) else (lambda k: getattr(o, k))
    cb = coef_bound(get("coefs"), cond, tol)
    cerr = np.abs(np.asarray(f.coefs) - get("coefs")) / np.maximum(np.abs(get("coefs")), 1e-300)
    serr = rel(f.stderr, get("stderr"))
    names = ("deviance", "null_deviance", "pearson", "loglik") if scalars else ()
    have = [n for n in names if (n in o if isinstance(o, dict) else hasattr(o, n))]
    verr = rel([getattr(f, n) for n in have], [get(n) for n in have]) if have else 0.0
    ratio = lambda bar, err: float(np.min(np.where(err > 0, bar / np.where(err > 0, err, 1.0), np.inf)))
    m_coef = ratio(cb, cerr)
    m_se, m_sc = ratio(tol, np.asarray(serr)), ratio(tol, np.asarray(verr))
    ill = bool(np.any(cb > tol))
    margin = min(m_coef, m_se, m_sc)
    print(f"\nMARGIN {label}: {margin:.3g} (coefs {m_coef:.3g} [{'cond-aware' if ill else f'fixed {tol:g}'}, cond "
          f"{cond:.2e}, max err {cerr.max():.2e}], stderr {m_se:.3g} [{serr:.2e}], scalars {m_sc:.3g} [{verr:.2e}])")
    if hasattr(f, "iter") and (isinstance(o, dict) and "iter" in o or hasattr(o, "iter")):
        assert f.iter == get("iter"), (label, f.iter, get("iter"))
    assert margin >= 1.0, (label, m_coef, m_se, m_sc)
    return margin
