"""The split-role narrow pass (narrow_r.hip irls_narrow_r_kernel: 64-row blocks in a workgroup-shared
LDS ring, four row waves -- LDS-DMA and the row stage with one row per lane -- and eight MFMA-only
Gram waves) against the oracle and against irls_narrow_kernel (SGLM_NARROW_SPLIT=0, read when an
engine is created).

The Gram waves accumulate other k-steps per wave than irls_narrow_kernel's waves and the row stage
forms eta in another order, so the two kernels are not bitwise: both are held to the oracle
(etaCreate / zwCreateBinomial / partitionComponents, GLM.scala:321-395, utils.scala:84-92) at 1e-9
with the same iteration count and to each other at ~1e-12 -- every family / link, offset + prior
weights, m, p = 33..64 (P16 = 3, 4; P16 = 2 forced), a shard whose last 64-row block holds only 32
rows of the image (an odd 32-row block count), one smaller than a block per workgroup, the LM Gram
and the deviance-only pass.  The split pass itself is deterministic: two runs bitwise equal."""
import os

import numpy as np
import pytest

from conftest import cond_ok, nrel, rel
from sparkglm_amd import Engine

pytestmark = pytest.mark.gpu


def _engine(split) -> Engine:
    saved = os.environ.get("SGLM_NARROW_SPLIT")
    os.environ["SGLM_NARROW_SPLIT"] = str(split)
    try:
        return Engine(0)
    finally:
        if saved is None:
            os.environ.pop("SGLM_NARROW_SPLIT", None)
        else:
            os.environ["SGLM_NARROW_SPLIT"] = saved


ODD = 32 * 6001 - 7  # 32-row block count 6001: the last 64-row block holds 32 rows of the image

CASES = [
    # (label, synth kind, rows, p, family, link, SGLM_NARROW_SPLIT)
    ("p64 poisson + offset + prior", 2, ODD, 64, "poisson", "log", 3),
    ("p40 poisson + offset + prior", 2, 150_000, 40, "poisson", "log", 3),
    ("p64 logit", 0, ODD, 64, "binomial", "logit", 3),
    ("p48 probit", 0, 120_001, 48, "binomial", "probit", 3),
    ("p57 cloglog", 0, 100_000, 57, "binomial", "cloglog", 3),
    ("p64 gamma", 3, 80_000, 64, "gamma", "inverse", 3),
    ("p36 gaussian", 1, 90_017, 36, "gaussian", "identity", 3),
    ("p33 logit (one column past a block pair)", 0, 70_000, 33, "binomial", "logit", 3),
    ("p32 logit (P16 = 2, forced)", 0, ODD, 32, "binomial", "logit", 2),
    ("p20 poisson + offset + prior (P16 = 2, forced)", 2, 100_000, 20, "poisson", "log", 2),
    ("p64 logit, fewer blocks than workgroups", 0, 3_000, 64, "binomial", "logit", 3),
    ("p20 gaussian, one block (P16 = 2, forced)", 1, 60, 20, "gaussian", "identity", 2),
]


@pytest.mark.parametrize("label,kind,n,p,family,link,ns", CASES, ids=[c[0] for c in CASES])
def test_split_and_classic_narrow_match_oracle(label, kind, n, p, family, link, ns):
    import pyoracle  # checker only
    fits = {}
    for split in (0, ns):
        with _engine(split) as e:
            e.synth(kind, 0, n, p, 17)
            f = e.fit_glm(family, link, init="multiple")
            kk = e.stats()["pass_kernel_kind"]
            if split:
                X, y, m, off, pr = e.get_data()
                cond = float(np.linalg.cond(e.irls_pass(f.coefs, family=family, link=link)[0]))
        assert kk == ("narrow-split" if split else "narrow"), (split, kk)
        fits[split] = f
    kw = dict(offset=off, prior=pr) if kind == 2 else {}
    o = pyoracle.fit_glm(X, y, family, link, nthreads=8, npart=2, **kw)
    for split, f in fits.items():
        assert f.iter == o.iter, (label, split)
        if family == "gamma":
            assert nrel(f.coefs, o.coefs) < 1e-9 and cond_ok(f.coefs, o.coefs, cond), (label, split, cond)
        else:
            assert rel(f.coefs, o.coefs) < 1e-9, (label, split)
        assert rel(f.stderr, o.stderr) < 1e-9, (label, split)
        assert rel([f.deviance, f.null_deviance, f.pearson, f.loglik],
                   [o.deviance, o.null_deviance, o.pearson, o.loglik]) < 1e-9, (label, split)
        assert rel(f.dev_trace, o.dev_trace) < 1e-9
    a, b = fits[0], fits[ns]  # the two kernels' Grams differ by summation order only
    assert (nrel if family == "gamma" else rel)(a.coefs, b.coefs) < 1e-10
    assert rel(a.stderr, b.stderr) < 1e-10 and rel(a.deviance, b.deviance) < 1e-12


def test_split_pass_is_deterministic_and_reports_its_kernel():
    beta = np.random.default_rng(3).normal(0.0, 0.05, 64)
    runs = []
    with _engine(3) as e:
        e.synth(2, 0, ODD, 64, 5)
        for _ in range(2):
            runs.append(e.irls_pass(beta, family="poisson", link="log"))
        st = e.stats()
    assert st["pass_kernel_kind"] == "narrow-split"
    assert st["pass_kernel_name"] == "irls_narrow_r_kernel<4,poisson,log>"
    for a, b in zip(*runs):
        assert np.array_equal(a, b)


def test_split_pass_gram_matches_classic_pass():
    # one pass at a fixed beta: X'WX, X'Wz and the scalars of the two narrow kernels
    beta = np.random.default_rng(9).normal(0.0, 0.05, 48)
    out = {}
    for split in (0, 3):
        with _engine(split) as e:
            e.synth(2, 0, 200_001, 48, 8)
            out[split] = e.irls_pass(beta, family="poisson", link="log")
    (g0, xz0, s0), (g1, xz1, s1) = out[0], out[3]
    assert rel(g1, g0) < 1e-12 and rel(xz1, xz0) < 1e-12
    assert rel(s1[:2], s0[:2]) < 1e-12


@pytest.mark.parametrize("p,ns", [(40, 3), (64, 3), (20, 2)])
def test_lm_fit_through_the_split_pass(p, ns):
    import pyoracle  # checker only
    n = 1_000_003
    with _engine(ns) as e:
        e.synth(1, 0, n, p, 1)
        f = e.fit_lm()
        assert e.stats()["pass_kernel_kind"] == "narrow-split"
        X, y, _, _, _ = e.get_data()
    r = pyoracle.fit_lm(X, y, nthreads=8)
    assert rel(f.coefs, r["coefs"]) < 1e-9 and rel(f.stderr, r["stderr"]) < 1e-9
    assert rel([f.sse, f.r2, f.fstat], [r["sse"], r["r2"], r["fstat"]]) < 1e-9


def test_speculative_deviance_pass_is_bitwise_the_full_pass():
    # the deviance-only pass (no Gram) carries the same row stage and scalar reduction
    fits = []
    for spec in ("1", "0"):
        saved = os.environ.get("SGLM_SPECULATE")
        os.environ["SGLM_SPECULATE"] = spec
        try:
            with _engine(3) as e:
                e.synth(2, 0, 300_000, 64, 21)
                fits.append((e.fit_glm("poisson", "log"), e.stats()["dev_passes"]))
        finally:
            if saved is None:
                os.environ.pop("SGLM_SPECULATE", None)
            else:
                os.environ["SGLM_SPECULATE"] = saved
    (a, da), (b, db) = fits
    assert da >= 1 and db == 0
    assert a.iter == b.iter and np.array_equal(a.coefs, b.coefs) and np.array_equal(a.stderr, b.stderr)
    assert (a.deviance, a.pearson, a.loglik) == (b.deviance, b.pearson, b.loglik)
