"""The split-role fused pass K1r (fused.hpp irls_pass_r_kernel: two MFMA-only "Gram waves" and
one "row wave" per SIMD) against K1 (irls_pass_kernel, SGLM_FUSED_SPLIT=0, read when an engine is
created).

At P16 = 16 (225 <= p <= 256) K1r accumulates every Gram tile and X'Wz column in K1's order (same
k-steps, blocks and lanes) and its row stage is K1's, so one pass and a whole fit must come out
BITWISE the same -- for every family / link and with offset + prior weights (the row stage's four
vectors, staged by the four row waves), at p = 256 and at p = 242 (column quads past p are
duplicated into the padded LDS image), over shards that split into ragged row ranges per
workgroup, and for a shard smaller than one row block per workgroup.

Below P16 = 16 (the mid-width generalisation, K1r by default from P16 = 10 and at every odd column-block
count from 9: p = 129..144, ..., 225..240 run ceil(p/16) blocks, where K1 runs the next even count;
odd 5 and 7 by SGLM_FUSED_SPLIT) the Gram waves own other tile runs than K1's waves and the row stage reads another lane layout
(and at odd counts the Gram itself is another tiling): NOT bitwise.  There both
kernels are held to the oracle (partitionComponents / zwCreateBinomial, GLM.scala:359-395,
utils.scala:84-92) at 1e-9 with the same iteration count, and to each other at 1e-12."""
import os

import numpy as np
import pytest

from sparkglm_amd import Engine

pytestmark = pytest.mark.gpu


def _engine(split: bool) -> Engine:
    saved = os.environ.get("SGLM_FUSED_SPLIT")
    os.environ["SGLM_FUSED_SPLIT"] = "1" if split else "0"
    try:
        return Engine(0)
    finally:
        if saved is None:
            os.environ.pop("SGLM_FUSED_SPLIT", None)
        else:
            os.environ["SGLM_FUSED_SPLIT"] = saved


CASES = [
    # (label, synth kind, rows, p, family, link)
    ("p256 logit", 0, 300_007, 256, "binomial", "logit"),
    ("p242 probit", 0, 150_001, 242, "binomial", "probit"),
    ("p248 cloglog", 0, 120_000, 248, "binomial", "cloglog"),
    ("p256 poisson + offset + prior", 2, 200_003, 256, "poisson", "log"),
    ("p250 gamma", 3, 100_000, 250, "gamma", "inverse"),
    ("p256 gaussian", 1, 90_000, 256, "gaussian", "identity"),
    ("p256 logit, fewer blocks than workgroups", 0, 5_000, 256, "binomial", "logit"),
]


@pytest.mark.parametrize("label,kind,n,p,family,link", CASES, ids=[c[0] for c in CASES])
def test_pass_and_fit_bitwise_k1(label, kind, n, p, family, link):
    rng = np.random.default_rng(p + n)
    beta = rng.normal(0.0, 0.02, p)
    if kind == 3:
        beta = np.abs(beta) + 0.01
        beta[0] = 1.0
    out = {}
    for split in (False, True):
        with _engine(split) as e:
            e.synth(kind, 0, n, p, 11)
            g, xz, s = e.irls_pass(beta, family=family, link=link)
            f = e.fit_glm(family, link)
            out[split] = (g, xz, s, f)
    (g0, xz0, s0, f0), (g1, xz1, s1, f1) = out[False], out[True]
    assert np.array_equal(g0, g1), label
    assert np.array_equal(xz0, xz1), label
    assert np.array_equal(s0, s1), label
    assert f0.iter == f1.iter
    assert np.array_equal(np.asarray(f0.coefs), np.asarray(f1.coefs))
    assert np.array_equal(np.asarray(f0.stderr), np.asarray(f1.stderr))
    assert (f0.deviance, f0.null_deviance, f0.pearson, f0.loglik) == (f1.deviance, f1.null_deviance, f1.pearson,
                                                                      f1.loglik)


MID = [
    # (label, synth kind, rows, p, family, link, K1r threshold SGLM_FUSED_SPLIT)
    ("p150 poisson + offset + prior", 2, 120_001, 150, "poisson", "log", "1"),
    ("p200 gamma", 3, 60_000, 200, "gamma", "inverse", "1"),
    ("p180 logit, fewer blocks than workgroups", 0, 3_000, 180, "binomial", "logit", "1"),
    ("p129 probit (odd P16 = 9)", 0, 90_000, 129, "binomial", "probit", "1"),
    ("p80 logit (odd P16 = 5, forced)", 0, 150_000, 80, "binomial", "logit", "5"),
    ("p70 poisson + offset + prior (odd P16 = 5, forced, padded stripe)", 2, 100_003, 70, "poisson", "log", "5"),
    ("p232 probit (odd P16 = 15)", 0, 90_001, 232, "binomial", "probit", "1"),
    ("p240 gaussian (odd P16 = 15)", 1, 60_000, 240, "gaussian", "identity", "1"),
    ("p105 gamma (odd P16 = 7, forced)", 3, 60_000, 105, "gamma", "inverse", "7"),
    ("p170 cloglog, few blocks (odd P16 = 11)", 0, 4_000, 170, "binomial", "cloglog", "1"),
    ("p96 cloglog, K1r forced from P16 = 6", 0, 100_000, 96, "binomial", "cloglog", "6"),
    ("p128 logit, K1r forced from P16 = 8", 0, 80_000, 128, "binomial", "logit", "8"),
    # the ring of up to four row-block buffers (GeoR::NBUF = 4 at P16 <= 8, 3 up to 12) partly filled:
    # fewer blocks than workgroups, and three blocks per workgroup
    ("p96 logit, fewer blocks than workgroups, 4-deep ring", 0, 5_000, 96, "binomial", "logit", "6"),
    ("p120 poisson + offset + prior, three blocks per workgroup, 4-deep ring", 2, 24_576, 120, "poisson", "log", "7"),
    ("p176 probit, two blocks per workgroup, 3-deep ring", 0, 16_384, 176, "binomial", "probit", "1"),
    ("p112 poisson + offset + prior, K1r forced from P16 = 6", 2, 80_000, 112, "poisson", "log", "6"),
]


@pytest.mark.parametrize("label,kind,n,p,family,link,thr", MID, ids=[c[0] for c in MID])
def test_mid_width_k1r_and_k1_match_oracle(label, kind, n, p, family, link, thr):
    import pyoracle  # checker only
    from conftest import cond_ok, nrel, rel
    fits = {}
    for split, env in (("K1", "0"), ("K1r", thr)):
        saved = os.environ.get("SGLM_FUSED_SPLIT")
        os.environ["SGLM_FUSED_SPLIT"] = env
        try:
            e = Engine(0)
        finally:
            if saved is None:
                os.environ.pop("SGLM_FUSED_SPLIT", None)
            else:
                os.environ["SGLM_FUSED_SPLIT"] = saved
        with e:
            e.synth(kind, 0, n, p, 13)
            f = e.fit_glm(family, link)
            kk = e.stats()["pass_kernel_kind"]
            if split == "K1r":
                X, y, m, off, pr = e.get_data()
                cond = float(np.linalg.cond(e.irls_pass(f.coefs, family=family, link=link)[0]))
        assert kk == ("fused" if split == "K1" else "fused-split"), (split, kk)
        fits[split] = f
    kw = dict(offset=off, prior=pr) if kind == 2 else {}
    o = pyoracle.fit_glm(X, y, family, link, nthreads=8, **kw)
    for split, f in fits.items():
        assert f.iter == o.iter, (label, split)
        # coefficients: 1e-9 elementwise, or -- gamma's ill-conditioned positive designs -- 1e-9
        # norm-wise and each within the solve's backward-error bound (conftest.cond_ok)
        if family == "gamma":
            assert nrel(f.coefs, o.coefs) < 1e-9 and cond_ok(f.coefs, o.coefs, cond), (label, split, cond)
        else:
            assert rel(f.coefs, o.coefs) < 1e-9, (label, split)
        assert rel(f.stderr, o.stderr) < 1e-9, (label, split)
        assert rel([f.deviance, f.null_deviance, f.pearson, f.loglik],
                   [o.deviance, o.null_deviance, o.pearson, o.loglik]) < 1e-9, (label, split)
        assert rel(f.dev_trace, o.dev_trace) < 1e-9
    a, b = fits["K1"], fits["K1r"]  # the two kernels' Grams differ by summation order only
    assert (nrel if family == "gamma" else rel)(a.coefs, b.coefs) < 1e-10
    assert rel(a.stderr, b.stderr) < 1e-10 and rel(a.deviance, b.deviance) < 1e-12


@pytest.mark.parametrize("p,name", [(160, "irls_pass_r_kernel<10,binomial,logit>"),
                                    (144, "irls_pass_r_kernel<9,binomial,logit>")])
def test_shard_reports_k1r(p, name):
    """The bench / roofline label comes from the engine's dispatch (sglm_stats.pass_kernel_name)."""
    with Engine(0) as e:
        e.synth(0, 0, 50_000, p, 3)
        e.irls_pass(np.full(p, 0.01))
        st = e.stats()
    assert st["pass_kernel_kind"] == "fused-split"
    assert st["pass_kernel_name"] == name
    assert st["kernel_variant"] == int(name.split("<")[1].split(",")[0])


def test_split_pass_matches_oracle():
    import pyoracle  # checker only
    n, p = 60_000, 256
    with _engine(True) as e:
        e.synth(2, 0, n, p, 5)
        X, y, m, off, pr = e.get_data()
        f = e.fit_glm("poisson", "log")
    o = pyoracle.fit_glm(X, y, "poisson", "log", offset=off, prior=pr, nthreads=8)
    rel = lambda a, b: float(np.max(np.abs(np.asarray(a) - b) / np.maximum(np.abs(b), 1e-300)))
    assert f.iter == o.iter
    assert rel(f.coefs, o.coefs) < 1e-9 and rel(f.stderr, o.stderr) < 1e-9
    assert rel(f.deviance, o.deviance) < 1e-9
