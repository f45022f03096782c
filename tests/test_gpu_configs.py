"""Every BASELINE.json config through the kernel variant its bench workload runs, against the
oracle -- at the bench's own full sizes where the streaming oracle pins them.

  configs[0]  LM.fit on the kind-1 1M x 20 design (narrow kernel, LM Gram mode)
  configs[1]  100M x 256 logit (fused pass irls_pass_kernel<16>)   -- full size, full_scale.json
  configs[2]  Poisson/log + offset + prior at p = 64 (irls_narrow_kernel<4>) -- 200k rows here,
              the 125M-row per-GPU shard at full size (full_scale.json)
  configs[3]  Gamma/inverse at p = 2048 (16 panels, rocSOLVER Cholesky)
  north star  1B x 32 logit on one GPU (irls_narrow_kernel<2>)     -- full size, full_scale.json

Bar (north_star): coefficients, standard errors, deviance within 1e-9 relative, identical
iteration count (LM: no iterations; coefs / stdErr / sse / r2 / F within 1e-9)."""
import json
import os

import numpy as np
import pytest

import pyoracle as po
from conftest import GOLDEN, nrel, rel
from sparkglm_amd import Engine, synth

pytestmark = pytest.mark.gpu
TOL = 1e-9


@pytest.fixture(scope="module")
def eng():
    e = Engine(0)
    yield e
    e.close()


def test_config0_lm_1m_x_20(eng):
    """BASELINE configs[0]: LM.fit (LM.scala:241-274) on the bench's own 1M x 20 design."""
    n, p = 1_000_000, 20
    eng.synth(1, 0, n, p, 1)
    X, y, _, _ = synth.generate(1, 0, n, p, 1)
    f = eng.fit_lm()
    st = eng.stats()
    assert st["path"] == 2 and st["kernel_variant"] == 2  # narrow kernel, P16 = 2
    r = po.fit_lm(X, y, nthreads=8)
    assert rel(f.coefs, r["coefs"]) < TOL and rel(f.stderr, r["stderr"]) < TOL
    assert rel([f.sse, f.r2, f.fstat, f.sigma], [r["sse"], r["r2"], r["fstat"], r["sigma"]]) < TOL
    assert rel(f.xtxi, r["xtxi"]) < 1e-8


def test_config2_poisson_offset_prior_p64(eng):
    """BASELINE configs[2]'s family / design / p through irls_narrow_kernel<4, poisson, log>."""
    n, p = 200_000, 64
    eng.synth(2, 5000, n, p, 3)
    X, y, off, pr = synth.generate(2, 5000, n, p, 3)
    f = eng.fit_glm("poisson", "log")
    st = eng.stats()
    assert st["path"] == 2 and st["kernel_variant"] == 4
    o = po.fit_glm(X, y, "poisson", "log", offset=off, prior=pr, nthreads=8)
    assert f.iter == o.iter
    assert rel(f.coefs, o.coefs) < TOL and rel(f.stderr, o.stderr) < TOL
    assert rel([f.deviance, f.null_deviance, f.pearson, f.loglik],
               [o.deviance, o.null_deviance, o.pearson, o.loglik]) < TOL
    assert rel(f.dev_trace, o.dev_trace) < TOL


def test_config3_gamma_p2048(eng):
    """BASELINE configs[3]'s family / design at p = 2048: all 16 column panels of the wide
    Gram kernel and the device (rocSOLVER) Cholesky + inverse, vs the oracle's LU inverse."""
    n, p = 6000, 2048
    eng.synth(3, 777, n, p, 4)
    f = eng.fit_glm("gamma", "inverse")
    st = eng.stats()
    assert st["path"] == 1 and st["wide_panels"] == 16
    o = po.fit_glm_synth(3, 777, n, p, 4, "gamma", "inverse", nthreads=16)
    assert f.iter == o.iter
    # cond(X'WX) ~1e6-1e7 here: the smallest coefficients (|b| ~ 0.03 beside max |b| ~ 11) move by
    # ~2e-9 relative under ANY change of solve algorithm -- Cholesky vs the reference's LU on the
    # oracle's own X'WX gives 1.85e-9 -- so coefficients are bounded norm-wise, the rest elementwise
    assert nrel(f.coefs, o.coefs) < TOL and rel(f.stderr, o.stderr) < TOL
    assert rel([f.deviance, f.null_deviance, f.pearson, f.loglik],
               [o.deviance, o.null_deviance, o.pearson, o.loglik]) < TOL


def _full_scale():
    path = os.path.join(GOLDEN, "full_scale.json")
    return json.load(open(path)) if os.path.exists(path) else {}


FULL = _full_scale()


@pytest.mark.parametrize("name", sorted(FULL))
def test_full_scale_fit_matches_streaming_oracle(eng, name):
    """The bench workloads at their full sizes (1B x 32, 100M x 256, 125M x 64 + offset + prior,
    and the wide ones: 60M x 512 logit -- overlapped row / Gram chunks -- and 12.5M x 2048 gamma
    with the GPU solve), generated in HBM, against the streaming oracle's fits of the same generator
    (tests/golden/make_full_scale.py): GLM.scala:452-462's absolute tol 1e-6 on a deviance of
    up to ~1.3e9 decides the iteration count, so the final |delta deviance| is printed beside it."""
    c = FULL[name]
    eng.synth(c["kind"], c["row0"], c["n"], c["p"], c["seed"])
    f = eng.fit_glm(c["family"], c["link"], tol=c["tol"])
    tr = np.asarray(c["dev_trace"])
    print(f"\n{name}: iter {f.iter} (oracle {c['iter']}); final |delta dev| engine "
          f"{abs(f.dev_trace[-1] - f.dev_trace[-2]):.3e} oracle {abs(tr[-1] - tr[-2]):.3e} vs tol {c['tol']:.0e}; "
          f"previous {abs(f.dev_trace[-2] - f.dev_trace[-3]):.3e}")
    assert f.iter == c["iter"]
    # gamma/inverse at p = 2048 is ill-conditioned: coefficients norm-wise
    ec = nrel(f.coefs, c["coefs"]) if c["family"] == "gamma" else rel(f.coefs, c["coefs"])
    assert ec < TOL and rel(f.stderr, c["stderr"]) < TOL, (ec, rel(f.stderr, c["stderr"]))
    assert rel([f.deviance, f.null_deviance, f.pearson, f.loglik],
               [c["deviance"], c["null_deviance"], c["pearson"], c["loglik"]]) < TOL
    assert rel(f.dev_trace, tr) < TOL
    eng.synth(c["kind"], 0, 64, c["p"], c["seed"])  # release the full-size shard
