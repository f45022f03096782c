"""Overlapped wide passes (engine.cpp enqueue_pass, resident X, p > 256): the rows are cut into
chunks; the row kernel of chunk c + 1 (eta = X beta + offset, zwCreate: GLM.scala:321-395) runs
on a second stream beside the Gram kernels of chunk c (partitionComponents / wlsComponents,
utils.scala:84-126), each chunk is reduced on its own and the chunks are summed in order -- the
same fixed-order treeReduce seam the multi-partition fit has.  The last chunk is shorter, so the
Gram kernels' clipped schedule runs too.  Checked against the oracle (1e-9, same iteration count),
against the non-overlapped engine, run to run bitwise, and with the speculative deviance-only pass
(bitwise the same fit)."""
import os

import numpy as np
import pytest

import pyoracle as po
from sparkglm_amd import Engine, synth

pytestmark = pytest.mark.gpu
TOL = 1e-9


def rel(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300)))


def nrel(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / np.max(np.abs(b)))


def _engine(chunks: int, spec: bool = True, devices=None) -> Engine:
    env = {"SGLM_WIDE_OVERLAP": str(chunks), "SGLM_WIDE_OV_MIN": "1024", "SGLM_SPECULATE": "1" if spec else "0"}
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return Engine(devices=devices) if devices else Engine(0)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def engines():
    e3, e1, e5 = _engine(3), _engine(1), _engine(5, spec=False)
    yield e3, e1, e5
    for e in (e3, e1, e5):
        e.close()


CASES = [  # (synth kind, rows, p, family, link)
    (0, 20000, 300, "binomial", "logit"),
    (2, 17000, 290, "poisson", "log"),
    (3, 9000, 520, "gamma", "inverse"),
    (0, 12000, 264, "binomial", "probit"),
]


@pytest.mark.parametrize("kind,n,p,fam,link", CASES)
def test_overlapped_pass_matches_oracle(engines, kind, n, p, fam, link):
    e3, e1, e5 = engines
    fits = []
    for e, want in ((e3, 3), (e1, 0), (e5, 5)):
        e.synth(kind, 500, n, p, 21)
        assert e.stats()["overlap_chunks"] == want
        fits.append(e.fit_glm(fam, link))
    f3, f1, f5 = fits
    X, y, off, pr = synth.generate(kind, 500, n, p, 21)
    kw = dict(offset=off, prior=pr) if kind == 2 else {}
    o = po.fit_glm(X, y, fam, link, nthreads=8, **kw)
    for f in (f3, f5):
        assert f.iter == o.iter == f1.iter
        # gamma/inverse designs are ill-conditioned: coefficients norm-wise there
        ec = nrel(f.coefs, o.coefs) if fam == "gamma" else rel(f.coefs, o.coefs)
        es = rel(f.stderr, o.stderr)
        assert ec < TOL and es < TOL, (ec, es)
        assert rel([f.deviance, f.null_deviance, f.pearson, f.loglik],
                   [o.deviance, o.null_deviance, o.pearson, o.loglik]) < TOL
        # another summation grouping than the one-launch pass: rounding-level differences only (the
        # LU inverse's diagonal carries them into stdErr at ~cond * eps: 1.06e-11 for gamma p = 520)
        d = (nrel(f.coefs, f1.coefs), rel(f.stderr, f1.stderr))
        assert d[0] < 1e-10 and d[1] < 1e-10, d


def test_overlapped_pass_is_deterministic_and_speculation_bitwise(engines):
    e3, _, _ = engines
    e3.synth(0, 0, 30000, 384, 5)
    a = e3.fit_glm("binomial", "logit")
    b = e3.fit_glm("binomial", "logit")
    assert e3.stats()["overlap_chunks"] == 3
    np.testing.assert_array_equal(a.coefs, b.coefs)
    np.testing.assert_array_equal(a.stderr, b.stderr)
    off = _engine(3, spec=False)
    try:
        off.synth(0, 0, 30000, 384, 5)
        c = off.fit_glm("binomial", "logit")
    finally:
        off.close()
    np.testing.assert_array_equal(a.coefs, c.coefs)
    np.testing.assert_array_equal(a.stderr, c.stderr)
    assert (a.deviance, a.pearson, a.loglik, a.iter) == (c.deviance, c.pearson, c.loglik, c.iter)
    np.testing.assert_array_equal(np.asarray(a.dev_trace), np.asarray(c.dev_trace))


def test_overlapped_lm_and_timing_split(engines):
    e3, _, _ = engines
    e3.synth(1, 0, 15000, 300, 9)
    e3.reset_stats()
    f = e3.fit_lm()
    X, y, _, _ = synth.generate(1, 0, 15000, 300, 9)
    r = po.fit_lm(X, y, nthreads=8)
    assert rel(f.coefs, r["coefs"]) < TOL and rel(f.stderr, r["stderr"]) < TOL
    st = e3.stats()
    assert st["row_kernel_ms"] > 0 and st["gram_kernel_ms"] > 0


def _proc_engine(chunks: int, spec: bool = True) -> Engine:
    env = {"SGLM_PROC_OVERLAP": str(chunks), "SGLM_PROC_OV_MIN": "4096", "SGLM_SPECULATE": "1" if spec else "0",
           "SGLM_WIDE_OVERLAP": "1"}
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return Engine(0)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("kind,p,fam,link", [(0, 520, "binomial", "logit"), (2, 300, "poisson", "log"),
                                              (2, 301, "poisson", "log"), (0, 263, "binomial", "logit")])
def test_overlapped_procedural_chunks(kind, p, fam, link):
    """Procedural shards (X generated per pass into an HBM scratch, configs[4]'s path) with two
    scratch buffers: chunk 0's generating row kernel, then for chunks >= 1 the lean generator
    (proc_gen_kernel: X and X beta, partial sums in the resident order) and the family stage from
    that eta, beside chunk c - 1's diagonal Gram launch.  Equal to the resident fit to rounding
    (another chunking) at p not a multiple of 4 too (the tail columns' partial sums), bitwise run
    to run and with the deviance-only last pass."""
    n = 30000
    ov, ov2, res = _proc_engine(6), _proc_engine(6, spec=False), _engine(1)
    try:
        ov.synth(kind, 77, n, p, 3, procedural=True)
        assert ov.stats()["overlap_chunks"] == 6
        a = ov.fit_glm(fam, link)
        b = ov.fit_glm(fam, link)
        ov2.synth(kind, 77, n, p, 3, procedural=True)
        c = ov2.fit_glm(fam, link)
        res.synth(kind, 77, n, p, 3)
        r = res.fit_glm(fam, link)
    finally:
        for e in (ov, ov2, res):
            e.close()
    np.testing.assert_array_equal(a.coefs, b.coefs)
    np.testing.assert_array_equal(a.coefs, c.coefs)
    np.testing.assert_array_equal(a.stderr, c.stderr)
    assert (a.deviance, a.pearson, a.loglik, a.iter) == (c.deviance, c.pearson, c.loglik, c.iter)
    assert a.iter == r.iter
    d = (rel(a.coefs, r.coefs), rel(a.stderr, r.stderr), rel([a.deviance, a.pearson], [r.deviance, r.pearson]))
    assert max(d) < 1e-11, d


def test_overlapped_shards_of_a_multi_device_handle():
    """One process over several devices (sglm_create_multi; here device 0 twice, host sums in
    shard order): every shard's pass overlaps its own row chunks with its Gram chunks."""
    g, one = _engine(3, devices=[0, 0]), _engine(1)
    try:
        g.synth(0, 0, 40000, 300, 17)
        assert g.stats()["overlap_chunks"] == 3
        f = g.fit_glm("binomial", "logit")
        one.synth(0, 0, 40000, 300, 17)
        r = one.fit_glm("binomial", "logit")
    finally:
        g.close()
        one.close()
    X, y, _, _ = synth.generate(0, 0, 40000, 300, 17)
    o = po.fit_glm(X, y, "binomial", "logit", nthreads=8)
    assert f.iter == o.iter == r.iter
    assert rel(f.coefs, o.coefs) < TOL and rel(f.stderr, o.stderr) < TOL
    assert rel(f.coefs, r.coefs) < 1e-11


def test_procedural_shards_of_a_multi_device_handle():
    """configs[4]'s procedural path (X generated per pass, never stored) sharded over the devices
    of one handle (here device 0 twice): the same fit as one device and as the oracle."""
    g, one = Engine(devices=[0, 0]), Engine(0)
    try:
        g.synth(0, 0, 20000, 520, 3, procedural=True)
        f = g.fit_glm("binomial", "logit")
        one.synth(0, 0, 20000, 520, 3, procedural=True)
        r = one.fit_glm("binomial", "logit")
    finally:
        g.close()
        one.close()
    X, y, _, _ = synth.generate(0, 0, 20000, 520, 3)
    o = po.fit_glm(X, y, "binomial", "logit", nthreads=8)
    assert f.iter == r.iter == o.iter
    assert rel(f.coefs, o.coefs) < TOL and rel(f.stderr, o.stderr) < TOL
    assert rel(f.coefs, r.coefs) < 1e-11 and rel([f.deviance], [r.deviance]) < 1e-12
