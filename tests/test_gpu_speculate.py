"""The speculative last pass of glm_drive (driver.cpp): when quadratic convergence predicts the
next |delta deviance| below tol / 10, the pass at the new beta runs without its Gram (which only a
further solve would read).  The deviance-only pass shares the full pass's row stage and scalar
reduction, so a fit must come out BITWISE identical with speculation on (default) and off
(SGLM_SPECULATE=0, read when an engine is created) -- on every kernel path -- and the counter
sglm_stats.dev_passes shows which fits took it.  (GLM.scala:452-462: the loop, its absolute tol
and the final statistics at the last mu.)"""
import os

import numpy as np
import pytest

from sparkglm_amd import Engine

pytestmark = pytest.mark.gpu


def _engine(spec: bool, force_wide: bool = False, devices=None) -> Engine:
    saved = {k: os.environ.get(k) for k in ("SGLM_SPECULATE", "SGLM_FORCE_WIDE")}
    os.environ["SGLM_SPECULATE"] = "1" if spec else "0"
    if force_wide:
        os.environ["SGLM_FORCE_WIDE"] = "1"
    try:
        return Engine(devices=devices) if devices else Engine(0)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _fit(e: Engine, kind, n, p, seed, family, link, procedural=False):
    e.synth(kind, 0, n, p, seed, procedural=procedural)
    e.reset_stats()
    f = e.fit_glm(family, link)
    return f, e.stats()["dev_passes"]


def _same(a, b):
    assert a.iter == b.iter
    assert np.array_equal(np.asarray(a.coefs), np.asarray(b.coefs))
    assert np.array_equal(np.asarray(a.stderr), np.asarray(b.stderr))
    assert (a.deviance, a.null_deviance, a.pearson, a.loglik) == (b.deviance, b.null_deviance, b.pearson, b.loglik)
    assert np.array_equal(np.asarray(a.dev_trace), np.asarray(b.dev_trace))


CASES = [
    # (label, synth kind, rows, p, family, link, force_wide, procedural)
    ("narrow p32 logit (stats in the pass)", 0, 400_000, 32, "binomial", "logit", False, False),
    ("narrow p20 probit", 0, 300_000, 20, "binomial", "probit", False, False),
    ("narrow p64 poisson + offset + prior", 2, 300_000, 64, "poisson", "log", False, False),
    ("fused p200 logit", 0, 200_000, 200, "binomial", "logit", False, False),
    ("fused p100 gamma", 3, 200_000, 100, "gamma", "inverse", False, False),
    ("wide p300 logit", 0, 100_000, 300, "binomial", "logit", False, False),
    ("forced-wide p40 cloglog", 0, 200_000, 40, "binomial", "cloglog", True, False),
    ("procedural p520 logit", 0, 50_000, 520, "binomial", "logit", False, True),
]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_speculative_last_pass_is_bitwise_the_full_pass(case):
    _, kind, n, p, fam, lnk, fw, proc = case
    on, off = _engine(True, fw), _engine(False, fw)
    try:
        f1, k1 = _fit(on, kind, n, p, 11, fam, lnk, proc)
        f0, k0 = _fit(off, kind, n, p, 11, fam, lnk, proc)
    finally:
        on.close()
        off.close()
    print(f"\n{case[0]}: iter {f1.iter}, deviance-only passes {k1}")
    assert k0 == 0
    assert k1 <= 2
    _same(f1, f0)


def test_speculation_taken_on_the_bench_shapes():
    """The headline's design (p = 256 logit) and the north star's (p = 32 logit) converge
    quadratically enough for the last pass to run without its Gram."""
    e = _engine(True)
    try:
        for p in (32, 256):
            f, k = _fit(e, 0, 1_000_000, p, 2, "binomial", "logit")
            assert k >= 1, (p, f.iter, f.dev_trace)
    finally:
        e.close()


def test_multi_device_handle_speculates_identically():
    on, off = _engine(True, devices=[0, 0]), _engine(False, devices=[0, 0])
    try:
        f1, k1 = _fit(on, 0, 300_000, 48, 7, "binomial", "logit")
        f0, k0 = _fit(off, 0, 300_000, 48, 7, "binomial", "logit")
    finally:
        on.close()
        off.close()
    assert k0 == 0
    _same(f1, f0)


@pytest.mark.parametrize("max_iter", [1, 2, 0])
def test_capped_fits_speculate_identically(max_iter):
    """A fit stopped by max_iter (GLM.scala has no cap; the engine's option) before any prediction
    is possible, or run to convergence, is bitwise the same with speculation on and off -- final
    statistics included (narrow binomial/logit: carried in every pass's scalars)."""
    on, off = _engine(True), _engine(False)
    try:
        res = []
        for e in (on, off):
            e.synth(0, 0, 300_000, 32, 5)
            e.reset_stats()
            res.append((e.fit_glm("binomial", "logit", max_iter=max_iter), e.stats()["dev_passes"]))
    finally:
        on.close()
        off.close()
    (f1, k1), (f0, k0) = res
    assert k0 == 0 and (k1 == 0 if max_iter else k1 >= 1)
    _same(f1, f0)


def test_default_overlapped_wide_pass_speculates_identically():
    """the overlapped wide pass at the DEFAULT chunking (SGLM_WIDE_OV_MIN = 65536 rows:
    >= 2 * ov_min rows give several chunks, the banded schedule over each) runs its deviance-only
    pass through the same chunk reduces -- bitwise the full pass's fit."""
    on, off = _engine(True), _engine(False)
    try:
        f1, k1 = _fit(on, 0, 262_144, 300, 13, "binomial", "logit")
        ch = on.stats()["overlap_chunks"]
        f0, k0 = _fit(off, 0, 262_144, 300, 13, "binomial", "logit")
    finally:
        on.close()
        off.close()
    print(f"\nwide p300 default chunks {ch}: iter {f1.iter}, deviance-only passes {k1}")
    assert ch >= 2 and k0 == 0 and k1 >= 1
    _same(f1, f0)
