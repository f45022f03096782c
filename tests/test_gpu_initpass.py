"""The initial (constant-mu) pass of a fit on the GPU (GLM.scala:263-272 fitSingle, 429-444
fitMultiple): its fast paths against the oracle's reference-order rows.

  * Poisson (narrow kernel, 32 < p <= 64): integer counts y < 256 take the per-workgroup LDS table
    of log(y / mu0), lgamma(y + 1) and y log y (rowmath.hpp poisson_init_table); every other row --
    fractional y, counts >= 256 -- the reference path.  Designs mixing both, with offset and prior
    weights, both init modes: the fit (iterations, coefficients, standard errors, deviance, null
    deviance, Pearson, loglik) against pyoracle at 1e-9;
  * binomial without m (fused K1 / K1r and narrow kernels): the constants at mu0 in LDS
    (init_const / pass_row_init) for 0 <= y <= 1, fractional proportions included."""
import numpy as np
import pytest

import pyoracle as po
from conftest import rel
from sparkglm_amd import Engine, synth

pytestmark = pytest.mark.gpu
TOL = 1e-9


@pytest.fixture(scope="module")
def eng():
    e = Engine(0)
    yield e
    e.close()


def _check(f, o):
    assert f.iter == o.iter
    assert rel(f.coefs, o.coefs) < TOL and rel(f.stderr, o.stderr) < TOL
    assert rel([f.deviance, f.null_deviance, f.pearson, f.loglik],
               [o.deviance, o.null_deviance, o.pearson, o.loglik]) < TOL


@pytest.mark.parametrize("p", [40, 64])
@pytest.mark.parametrize("init", ["single", "multiple"])
def test_poisson_init_table_and_fallback_rows(eng, p, init):
    n = 120_011
    X, y, off, prior = synth.generate(2, 0, n, p, 31)
    rng = np.random.default_rng(p)
    y = y.copy()
    frac = rng.random(n) < 0.05            # fractional counts: reference path
    y[frac] += 0.375
    big = rng.random(n) < 0.02             # counts beyond the table
    y[big] = 256.0 + np.floor(rng.random(big.sum()) * 40.0)
    assert (y == np.floor(y)).mean() > 0.9 and (y >= 256).any()
    eng.set_data(X, y, offset=off, prior=prior)
    f = eng.fit_glm("poisson", "log", init=init)
    o = po.fit_glm(X, y, "poisson", "log", offset=off, prior=prior, nthreads=8,
                   npart=1 if init == "single" else 4)
    _check(f, o)


@pytest.mark.parametrize("p", [48, 128, 256])
def test_binomial_init_fractional_proportions(eng, p):
    n = 90_007
    X, y, _, _ = synth.generate(0, 0, n, p, 17)
    rng = np.random.default_rng(p)
    y = y.copy()
    part = rng.random(n) < 0.3
    y[part] = np.round(rng.random(part.sum()) * 8.0) / 8.0  # proportions in [0, 1]
    eng.set_data(X, y)
    f = eng.fit_glm("binomial", "logit", init="multiple")
    o = po.fit_glm(X, y, "binomial", "logit", nthreads=8, npart=4)
    _check(f, o)
