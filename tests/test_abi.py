"""The C-ABI library: loads on a CPU-only host, exports every symbol include/sglm.h
declares, and its host-side logic (driver over external partials, solves, summaries)
agrees with the oracle.  No GPU calls."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import pyoracle as po
from conftest import ROOT, iris_design, rel
from sparkglm_amd import _lib as L
from sparkglm_amd import distributed as D


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "sglm.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sglm_[a-z0-9_]+)\s*\(", src)) - {"sglm_allreduce_fn"})


def test_library_exports_every_declared_symbol():
    lib = L.load()
    syms = declared_symbols()
    assert len(syms) >= 29
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(L.EXPORTS) == syms
    assert lib.sglm_abi_version() == 8


def test_java_double_to_string():
    cases = {1.0: "1.0", 3.8443: "3.8443", 0.001: "0.001", 1e-4: "1.0E-4", 1e7: "1.0E7", 1234567.0: "1234567.0",
             -0.5: "-0.5", 145.0: "145.0", 0.0: "0.0", float("nan"): "NaN", float("inf"): "Infinity",
             2.5e-10: "2.5E-10", 123456789.0: "1.23456789E8", 0.1 + 0.2: "0.30000000000000004"}
    for x, s in cases.items():
        assert L.java_double_str(x) == s, (x, L.java_double_str(x))


def test_sig_and_round_digits():
    lib = L.load()
    assert lib.sglm_sig_digits(3.14159265, 3) == 3.14
    assert lib.sglm_sig_digits(-0.000123456, 2) == -0.00012
    assert lib.sglm_sig_digits(0.0, 6) == 0.0
    assert lib.sglm_round_digits(3.844317270060284, 4) == 3.8443
    assert lib.sglm_round_digits(3.9227811947516025, 4) == 3.9228
    assert abs(lib.sglm_pval_normal(1.959963984540054) - 0.05) < 1e-12
    from scipy import stats
    for t, df in ((2.0, 5.0), (0.3, 145.0), (4.5, 30.0)):
        assert abs(lib.sglm_pval_t(t, df) - 2 * stats.t.sf(t, df)) < 1e-12


def _ext_fit(c, **kw):
    X, y = c["X"], c["y"]
    fam, link = (str(v) for v in c["meta"][:2])
    m, off, pr = c.get("m"), c.get("offset"), c.get("prior")
    sums = lambda: (y.sum(), len(y))
    part = lambda mode, b, mu0, ybar: po.shard_partials(X, y, fam, link, mode, b, mu0, ybar, m=m, offset=off, prior=pr)
    return D.fit_glm_external(X.shape[1], sums, part, family=fam, link=link, **kw)


def test_driver_over_external_partials_matches_oracle(golden):
    for name, c in golden.items():
        if str(c["meta"][2]) != "1":
            continue
        f = _ext_fit(c)
        s = c["scalars"]
        assert f.iter == int(s[4]), name
        if np.isnan(s[0]):
            assert np.isnan(f.deviance)
            continue
        assert rel(f.coefs, c["coefs"]) < 1e-9, name
        assert rel(f.stderr, c["stderr"]) < 1e-9, name
        assert rel([f.deviance, f.null_deviance, f.pearson, f.loglik], s[:4]) < 1e-9, name


def test_driver_multi_init_matches_partitioned_oracle(golden):
    c = golden["logit_npart4"]
    f = _ext_fit(c, init="multiple", npart=4)
    assert f.iter == int(c["scalars"][4]) and f.npart == 4
    assert rel(f.coefs, c["coefs"]) < 1e-9 and rel(f.stderr, c["stderr"]) < 1e-9


def test_lm_driver_and_summary_reproduce_reference_r2_string(iris):
    X, y, names = iris_design(iris)
    part = lambda mode, b, mu0, ybar: po.shard_partials(X, y, "gaussian", "identity", mode, b, mu0, ybar)
    f = D.fit_lm_external(X.shape[1], lambda: (y.sum(), len(y)), part)
    r = po.fit_lm(X, y)
    assert rel(f.coefs, r["coefs"]) < 1e-10 and rel(f.stderr, r["stderr"]) < 1e-10
    lib = L.load()
    coefs, se = np.ascontiguousarray(f.coefs), np.ascontiguousarray(f.stderr)
    pre = L.PreLM(L.ptr(coefs), None, L.ptr(se), f.sse, f.r2, f.fstat, f.sigma, f.nrow, 1)
    cn = (C.c_char_p * 4)(*[n.encode() for n in names])
    buf = C.create_string_buffer(4096)
    lib.sglm_lm_summary(C.byref(pre), 4, cn, b"Sepal_Width", buf, 4096)
    text = buf.value.decode()
    # R/pkg/tests/testthat/test_LM.R:44
    assert "Multiple R-Squared: 3.8443, Adusted R-Squared: 3.9228" in text
    assert "Sepal_Width ~ Petal_Length + Petal_Width + Species_versicolor + Species_virginica" in text
    assert "on 146.0 degrees of freedom" in text


def test_unsupported_family_link_raises_illegal_argument(golden):
    c = golden["logit"]
    with pytest.raises(L.IllegalArgumentException):
        D.fit_glm_external(5, lambda: (1.0, 2.0), lambda *a: np.zeros(5 * 6 // 2 + 5 + 8), family="poisson",
                           link="logit")


def test_singular_gram_raises_matrix_singular():
    X = np.ones((40, 2))  # duplicated column: X'X exactly singular
    y = np.arange(40.0)
    part = lambda mode, b, mu0, ybar: po.shard_partials(X, y, "gaussian", "identity", mode, b, mu0, ybar)
    with pytest.raises(L.MatrixSingularException):
        D.fit_lm_external(2, lambda: (y.sum(), 40), part)


def test_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from sparkglm_amd import Engine
    with pytest.raises(L.SGLMError):
        Engine(0)


def test_create_takes_a_device_list_and_refuses_bad_arguments():
    """SURVEY 8(b)'s constructor sglm_create(const int* devs, int ndev, ...): the requires fail with
    SGLM_EINVAL before any device is touched; on a host without a GPU a valid list fails with
    SGLM_EHIP (loudly, no CPU fallback)."""
    lib = L.load()
    h = C.c_void_p()
    devs = (C.c_int * 2)(0, 0)
    assert lib.sglm_create(None, 1, C.byref(h)) == 1 and not h.value
    assert lib.sglm_create(devs, 0, C.byref(h)) == 1
    assert lib.sglm_create(devs, 1, None) == 1
    assert lib.sglm_create_multi(devs, 0, C.byref(h)) == 1
    import torch
    if not torch.cuda.is_available():
        assert lib.sglm_create(devs, 1, C.byref(h)) == 3 and not h.value
        assert lib.sglm_create_device(0, C.byref(h)) == 3


def test_integration_knob_table_equals_the_getenv_list():
    """Every environment knob the engine reads (getenv in csrc/) is documented in INTEGRATION.md's
    runtime-knob table, and the table lists no knob the engine no longer reads."""
    src = ""
    for f in os.listdir(os.path.join(ROOT, "sparkglm_amd", "csrc")):
        if f.endswith((".cpp", ".hpp", ".hip")):
            src += open(os.path.join(ROOT, "sparkglm_amd", "csrc", f)).read()
    read = set(re.findall(r'getenv\("(SGLM_[A-Z0-9_]+)"\)', src))
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    table = doc[doc.index("## Runtime knobs"):]
    rows = set(re.findall(r"^\| `(SGLM_[A-Z0-9_]+)`(?:, `(SGLM_[A-Z0-9_]+)`)?", table, flags=re.M))
    listed = {k for r in rows for k in r if k} - {"SGLM_LIB"}  # SGLM_LIB: the Python mirror's, not the engine's
    assert read == listed, (read - listed, listed - read)
