"""Poisson / log with LARGE counts through the narrow pass (p <= 64), at a row count where the
deviance's rounding matters for GLM.scala:452's absolute tol 1e-6 on its change.

The narrow kernel's Poisson rows sum the unit deviance y log(y / mu) - (y - mu) per row (rowmath.hpp
pass_row: y log y from an LDS table for integer counts below POIS_TAB = 256, log_pos above), so every
term is of the size of its row's own deviance.  A round-3 form summed -y eta - (y - mu) per row and
added sum y log y once: with counts ~1e3 over 2e7 rows its terms reach ~1e11 and their rounding
(~1e-5) exceeds tol, so the iteration count and the deviance trajectory followed the summation noise
instead of the fit.  Here the fit must match the oracle's (orc_fit_glm, per-row reference order)
iteration count and whole deviance trajectory at 1e-9, for counts in the table (~80) and above it
(~1000).  Data: numpy-seeded Poisson draws (parity unpinned by the reference, which has no Poisson
family: SURVEY 8a-ext)."""
import numpy as np
import pytest

import pyoracle as po
from conftest import rel
from sparkglm_amd import Engine

pytestmark = pytest.mark.gpu


def _design(n, p, level, seed):
    rng = np.random.default_rng(seed)
    X = np.empty((n, p), order="F")
    X[:, 0] = 1.0
    X[:, 1:] = rng.uniform(-1.0, 1.0, size=(n, p - 1))
    b = np.zeros(p)
    b[0] = np.log(level)
    b[1:] = rng.uniform(-0.05, 0.05, size=p - 1)
    y = rng.poisson(np.exp(X @ b)).astype(np.float64)
    return X, y


@pytest.mark.parametrize("level,in_table", [(80.0, True), (1000.0, False)])
def test_large_count_poisson_matches_oracle_trajectory(level, in_table):
    n, p = 20_000_000, 16
    X, y = _design(n, p, level, 7 + int(level))
    assert (y.max() < 256) == in_table  # every count in the LDS table (or none of them)
    with Engine(0) as e:
        e.set_data(X, y)
        f = e.fit_glm("poisson", "log")
        st = e.stats()
    assert st["pass_kernel_kind"] == "narrow"
    o = po.fit_glm(X, y, "poisson", "log", nthreads=16)
    d = np.diff(np.asarray(f.dev_trace))
    print(f"\ncounts ~{level:.0f} (max {y.max():.0f}): iter {f.iter} (oracle {o.iter}); delta dev {d.tolist()}")
    assert f.iter == o.iter
    assert rel(f.dev_trace, o.dev_trace) < 1e-9
    assert rel(f.coefs, o.coefs) < 1e-9 and rel(f.stderr, o.stderr) < 1e-9
    assert rel([f.deviance, f.null_deviance, f.pearson, f.loglik], [o.deviance, o.null_deviance, o.pearson, o.loglik]) < 1e-9
