"""Generates tests/golden/glm_golden.npz: inputs and oracle outputs for the GLM/LM cases.

The reference holds no numeric GLM expectations (its GLM has no tests), so
these vectors are produced by the CPU restatement (oracle/) -- after it has been checked
against the reference's one known answer (iris R^2, test_LM.R:44) and against independent
numpy/scipy/sklearn fits (tests/test_oracle.py).  They pin the restatement against
regressions and serve the GPU parity tests.  Inputs come from the documented counter-based
generator (sparkglm_amd.synth), so nothing here depends on a numpy RNG version.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle  # noqa: E402
from sparkglm_amd import synth  # noqa: E402


def u(seed, n):
    return synth.unif(np.uint64(synth._sm_scalar(seed)) + np.arange(n, dtype=np.uint64))


def cases():
    out = {}
    # binomial / logit, synthetic design kind 0 (the bench generator)
    X, y, _, _ = synth.generate(0, 0, 600, 5, 11)
    out["logit"] = dict(X=X, y=y, family="binomial", link="logit")
    X, y, _, _ = synth.generate(0, 1000, 700, 5, 12)
    out["logit_npart4"] = dict(X=X, y=y, family="binomial", link="logit", npart=4)
    # probit / cloglog with a stronger signal: y ~ Bernoulli(Phi(eta)) by thresholding u
    X, _, _, _ = synth.generate(0, 0, 800, 8, 13)
    eta = X @ (0.8 * synth.beta_star(8))
    from scipy.special import ndtr
    y = (u(99, 800) < ndtr(eta)).astype(float)
    out["probit"] = dict(X=X, y=y, family="binomial", link="probit")
    X, _, _, _ = synth.generate(0, 0, 1000, 6, 14)
    eta = X @ (0.5 * synth.beta_star(6)) - 0.5
    y = (u(98, 1000) < 1 - np.exp(-np.exp(eta))).astype(float)
    out["cloglog"] = dict(X=X, y=y, family="binomial", link="cloglog")
    # grouped binomial: m trials per row and an offset (fitSingle with offset + m overloads)
    X, _, _, _ = synth.generate(0, 0, 500, 4, 15)
    m = 1.0 + np.floor(u(97, 500) * 5.0)
    pr = 1 / (1 + np.exp(-(X @ synth.beta_star(4))))
    y = np.floor(m * pr + u(96, 500))
    y = np.minimum(y, m)
    off = 0.1 * (2 * u(95, 500) - 1)
    # the reference starts every row at mu = mean(y) (GLM.scala:263), so rows with m < mean(y)
    # give log(negative) = NaN: the fit stops after one iteration with a NaN deviance.
    out["binomial_m_quirk"] = dict(X=X, y=y, m=m, offset=off, family="binomial", link="logit")
    m2 = 4.0 + np.floor(u(93, 500) * 3.0)
    y2 = np.minimum(np.floor(m2 * 0.6 * pr + u(92, 500)), m2)
    out["binomial_m_offset"] = dict(X=X, y=y2, m=m2, offset=off, family="binomial", link="logit")
    # extension families (no reference implementation; R family formulas)
    X, y, off, prior = synth.generate(2, 0, 800, 5, 16)
    out["poisson_offset_prior"] = dict(X=X, y=y, offset=off, prior=prior, family="poisson", link="log")
    X, _, _, _ = synth.generate(0, 0, 600, 4, 17)
    X[:, 1:] = 0.5 + np.abs(X[:, 1:])
    mu = 1.0 / (X @ np.array([0.5, 0.3, 0.2, 0.4]))
    y = mu * (-np.log(1 - u(94, 600)))  # exponential (gamma shape 1)
    out["gamma"] = dict(X=X, y=y, family="gamma", link="inverse")
    X, y, _, _ = synth.generate(1, 0, 500, 6, 18)
    out["gaussian"] = dict(X=X, y=y, family="gaussian", link="identity")
    return out


def main():
    arrays = {}
    for name, c in cases().items():
        f = pyoracle.fit_glm(c["X"], c["y"], c["family"], c["link"], m=c.get("m"), offset=c.get("offset"),
                             prior=c.get("prior"), npart=c.get("npart", 1), nthreads=1)
        for k in ("X", "y", "m", "offset", "prior"):
            if c.get(k) is not None:
                arrays[f"{name}/{k}"] = np.asarray(c[k])
        arrays[f"{name}/meta"] = np.array([c["family"], c["link"], str(c.get("npart", 1))])
        arrays[f"{name}/coefs"] = f.coefs
        arrays[f"{name}/stderr"] = f.stderr
        arrays[f"{name}/scalars"] = np.array([f.deviance, f.null_deviance, f.pearson, f.loglik, f.iter, f.nrow])
        arrays[f"{name}/trace"] = f.dev_trace
        print(f"{name:22s} iter={f.iter} dev={f.deviance:.10g}")
    np.savez_compressed(os.path.join(HERE, "glm_golden.npz"), **arrays)


if __name__ == "__main__":
    main()
