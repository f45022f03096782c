"""An independent numpy/scipy restatement of the reference's IRLS, written straight from the Scala.

TEST INFRASTRUCTURE ONLY (imported by tests/, never by sparkglm_amd).  It cross-checks the C
oracle (oracle/sglm_oracle.c), which shares its author with the HIP kernels: a misreading common
to both would pass every GPU parity test, so this file restates the reference a second time,
vectorised the way Breeze evaluates it, with none of the C oracle's code:

  * the Breeze expressions of GLM.scala:90-251 elementwise over whole vectors (numpy);
  * Breeze `inv` as LAPACK dgetrf + dgetri (scipy.linalg.lapack: the routines netlib-java binds),
    `coefs = XtWXi * XtWy`, `diagDesign = sqrt(diag(XtWXi))` (utils.scala:98-107, 129-138);
  * `leftMultDiag(X.t, w)` then `XtW * X`, `XtW * y` as BLAS products (utils.scala:68-92);
  * the deviance as the ones-vector product of devBinomial (GLM.scala:162-170), partitions summed
    in partition order (GLM.scala:397-408);
  * Breeze Gaussian(0, 1) from its published definitions (icdf = sqrt(2) erfinv(2p - 1), cdf =
    (1 + erf(x / sqrt 2)) / 2, pdf = exp(-x^2 / 2) / sqrt(2 pi)) via scipy.special;
  * Breeze Binomial(n, p).logProbabilityOf(k) as scipy.stats.binom.logpmf with GLM.scala:140's
    `m.toInt` / `y.toInt` truncations and p = mu (its quirk).

The extension families (Gaussian / Poisson / Gamma GLM, prior weights; not in the reference,
SURVEY.md 8(a-ext)) follow R's family objects on the same skeleton: R's variance, link, deviance
residuals and aic() log-likelihoods (scipy.stats for the densities).

  fit_glm(X, y, family, link, m=None, offset=None, prior=None, tol=1e-6, npart=1)
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import scipy.linalg.lapack as lapack
from scipy import special, stats

SQRT2 = np.sqrt(2.0)


# ---- Breeze Gaussian(0, 1) (GLM.scala:212, 222, 231) ----
def g_icdf(q):
    return 0.0 + 1.0 * SQRT2 * special.erfinv(2.0 * q - 1.0)


def g_cdf(x):
    return 0.5 * (1.0 + special.erf(x / SQRT2))


def g_pdf(x):
    return np.exp(-0.5 * x * x) / np.sqrt(2.0 * np.pi)


# ---- binomial links (GLM.scala:190-251) ----
def link(family, lnk, mu, m):
    if family == "binomial":
        if lnk == "logit":
            return np.log(mu / (m + (-1.0 * mu)))                      # GLM.scala:193
        if lnk == "probit":
            return g_icdf(mu / m)                                       # GLM.scala:212
        return np.log(-1.0 * np.log(1.0 + (-1.0 * (mu / m))))         # GLM.scala:240
    if family == "gaussian":
        return mu
    if family == "poisson":
        return np.log(mu)
    return 1.0 / mu                                                     # gamma / inverse


def lprime(family, lnk, mu, m):
    if family == "binomial":
        if lnk == "logit":
            return m / (mu * (m + (-1.0 * mu)))                         # GLM.scala:198
        if lnk == "probit":
            return 1.0 / (m * g_pdf(g_icdf(mu / m)))                   # GLM.scala:215-223
        return 1.0 / ((mu + (-1.0 * m)) * np.log(1.0 + (-1.0 * (mu / m))))  # GLM.scala:245
    if family == "gaussian":
        return np.ones_like(mu)
    if family == "poisson":
        return 1.0 / mu
    return -1.0 / (mu * mu)


def unlink(family, lnk, eta, m):
    if family == "binomial":
        if lnk == "logit":
            return m / (1.0 + np.exp(-1.0 * eta))                       # GLM.scala:203
        if lnk == "probit":
            return m * g_cdf(eta)                                       # GLM.scala:231
        return m * (1.0 + (-1.0 * np.exp(-np.exp(eta))))               # GLM.scala:250
    if family == "gaussian":
        return eta
    if family == "poisson":
        return np.exp(eta)
    return 1.0 / eta


def variance(family, mu, m):
    if family == "binomial":
        return mu * (1.0 + (-1.0 * (mu / m)))                           # GLM.scala:128
    if family == "gaussian":
        return np.ones_like(mu)
    if family == "poisson":
        return mu
    return mu * mu


def dev_rows(family, y, mu, m, pw):
    """Unit deviances (family factor applied by the caller): devBinomial's rowValue
    (GLM.scala:166-167); R's dev.resids for the extension families."""
    with np.errstate(divide="ignore", invalid="ignore"):
        if family == "binomial":
            my = m + (-1.0 * y)
            return pw * ((y * np.log(np.maximum(y, 1.0) / mu)) + (my * np.log(np.maximum(my, 1.0) / (m + (-1.0 * mu)))))
        if family == "gaussian":
            return pw * (y - mu) ** 2
        if family == "poisson":
            ylogy = np.where(y > 0, y * np.log(np.where(y > 0, y, 1.0) / mu), 0.0)
            return pw * (ylogy - (y - mu))
        return pw * (-(np.log(y / mu) - (y - mu) / mu))


def dev_factor(family):
    return 1.0 if family == "gaussian" else 2.0


def parts(n, G):
    """Spark's ParallelCollectionRDD slicing [g n / G, (g + 1) n / G)."""
    return [((g * n) // G, ((g + 1) * n) // G) for g in range(G)]


def deviance(family, y, mu, m, pw, G):
    """createBinomialDeviance (GLM.scala:397-408): per partition the ones-vector product
    (GLM.scala:168), the partition values reduced in partition order."""
    tot = 0.0
    for a, b in parts(len(y), G):
        r = dev_rows(family, y[a:b], mu[a:b], m[a:b], pw[a:b])
        tot = tot + dev_factor(family) * float(np.ones(b - a) @ r)
    return tot


def breeze_inv(A):
    """Breeze inv(): LAPACK dgetrf + dgetri (utils.scala:103, 134).  A zero pivot is
    breeze.linalg.MatrixSingularException."""
    lu, piv, info = lapack.dgetrf(A)
    if info > 0:
        raise np.linalg.LinAlgError("MatrixSingularException")
    inv, info = lapack.dgetri(lu, piv)
    if info != 0:
        raise np.linalg.LinAlgError("MatrixSingularException")
    return inv


def wls(X, z, w, G):
    """wlsSingle / wlsMultiple (utils.scala:98-107, 110-138): per partition leftMultDiag(X.t, w)
    (utils.scala:68-80), XtW * X and XtW * y (:89-90), the partitions reduced by reduceNormal
    (:58-64); inv, coefs = XtWXi * XtWy, diagDesign = sqrt(diag(XtWXi))."""
    p = X.shape[1]
    XtWX, XtWy = np.zeros((p, p)), np.zeros(p)
    for a, b in parts(X.shape[0], G):
        XtW = X[a:b].T * w[a:b]
        XtWX = XtWX + XtW @ X[a:b]
        XtWy = XtWy + XtW @ z[a:b]
    XtWXi = breeze_inv(XtWX)
    return XtWXi @ XtWy, np.sqrt(np.diag(XtWXi))


def loglik(family, y, mu, m, pw, dev):
    """llBinomial (GLM.scala:132-159): Binomial(m.toInt, mu).logProbabilityOf(y.toInt) -- with
    mu, not mu / m, as the probability (the reference's quirk); R's aic() log-likelihoods for the
    extension families."""
    with np.errstate(divide="ignore", invalid="ignore"):
        if family == "binomial":
            n, k = np.trunc(m).astype(np.int64), np.trunc(y).astype(np.int64)
            pr = np.where((mu >= 0) & (mu <= 1), mu, np.nan)
            return float(np.sum(pw * stats.binom.logpmf(k, n, pr)))
        if family == "poisson":
            return float(np.sum(pw * stats.poisson.logpmf(y, mu))) if np.all(y == np.floor(y)) else float(
                np.sum(pw * (y * np.log(mu) - mu - special.gammaln(y + 1.0))))
        nobs = len(y)
        if family == "gaussian":
            return float(-(nobs / 2.0) * (np.log(2.0 * np.pi * dev / nobs) + 1.0) + 0.5 * np.sum(np.log(pw)))
        disp = dev / np.sum(pw)
        return float(np.sum(pw * stats.gamma.logpdf(y, 1.0 / disp, scale=mu * disp)))


@dataclass
class Fit:
    coefs: np.ndarray
    stderr: np.ndarray
    deviance: float
    null_deviance: float
    pearson: float
    loglik: float
    iter: int
    dev_trace: np.ndarray


def fit_glm(X, y, family="binomial", lnk="logit", m=None, offset=None, prior=None, tol=1e-6, npart=1,
            max_iter=0) -> Fit:
    """fitSingleBinomial (GLM.scala:254-315) for npart == 1, fitMultipleBinomial (:410-468) over
    npart row partitions otherwise (mu re-derived as unlink(eta) inside zwCreateBinomial,
    :359-395).  No iteration cap unless max_iter > 0 (the reference has none)."""
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    n = len(y)
    m = np.ones(n) if m is None else np.asarray(m, dtype=np.float64)
    off = np.zeros(n) if offset is None else np.asarray(offset, dtype=np.float64)
    pw = np.ones(n) if prior is None else np.asarray(prior, dtype=np.float64)
    G = max(int(npart), 1)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        ysum = 0.0
        for a, b in parts(n, G):  # GLM.scala:263 (single) / 420-423 (per-partition sums, reduced)
            ysum = ysum + float(np.sum(y[a:b]))
        mu = np.full(n, ysum / n)
        eta = link(family, lnk, mu, m)                               # offset ignored: GLM.scala:264-270
        dev = deviance(family, y, mu, m, pw, G)                      # GLM.scala:271 / 443
        null_dev, deltad, it = dev, 1.0, 0
        trace = [dev]
        coefs, se = np.zeros(X.shape[1]), np.zeros(X.shape[1])
        while abs(deltad) > tol:                                     # GLM.scala:281 / 452 (NaN ends it)
            if max_iter and it >= max_iter:
                break
            mz = mu if G == 1 else unlink(family, lnk, eta, m)       # GLM.scala:282-290 / 370-371
            grad = lprime(family, lnk, mz, m)
            w = pw * (1.0 / (variance(family, mz, m) * grad ** 2))   # GLM.scala:289
            z = eta + ((y + (-1.0 * mz)) * grad) + (-1.0 * off)       # GLM.scala:290
            coefs, se = wls(X, z, w, G)
            eta = (X @ coefs) + off                                  # GLM.scala:292 / 321-332
            mu = unlink(family, lnk, eta, m)                         # GLM.scala:293-299 / 334-355
            dev_old, dev = dev, deviance(family, y, mu, m, pw, G)
            deltad = dev - dev_old
            it += 1
            trace.append(dev)
        pear = 0.0
        for a, b in parts(n, G):  # pearsonCalc(Multiple) (GLM.scala:90-118): binomial variance
            r = y[a:b] + (-1.0 * mu[a:b])
            pear = pear + float(np.sum(pw[a:b] * r ** 2 / variance(family, mu[a:b], m[a:b])))
        ll = loglik(family, y, mu, m, pw, dev)
    return Fit(coefs, se, dev, null_dev, pear, ll, it, np.array(trace))
