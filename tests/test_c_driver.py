"""The C-ABI boundary driven from plain C (tests/c_abi/sglm_c_driver.c, C99, gcc -Wall -Wextra -Werror
-pedantic against include/sglm.h): SURVEY 8(b)'s "C-ABI exercised by a C++ test driver and Python
ctypes tests".  The driver does what a JNI binding does -- no Python between it and the library --
and prints its results; they are checked here against the oracle (LM.scala:142-274,
GLM.scala:254-315).

  cpu: LM.fit over caller-computed partials (sglm_fit_lm_external) on two threads joined by the
       in-process communicator, the SummaryLM text, and the requires / no-device errors
  gpu: sglm_create(devs, 1), set_data, fit_glm, predict_new, the GLM summary, fit_lm on device 0"""
import os
import shutil
import subprocess

import numpy as np
import pytest

import pyoracle as po
from conftest import ROOT, rel
from sparkglm_amd import synth

DRIVER_DIR = os.path.join(ROOT, "tests", "c_abi")
DRIVER = os.path.join(DRIVER_DIR, "build", "sglm_c_driver")


def _driver():
    if not os.path.exists(DRIVER):
        if not shutil.which(os.environ.get("CC", "gcc")):
            pytest.skip("no C compiler")
        subprocess.run(["make", "-s", "-C", DRIVER_DIR], check=True, capture_output=True, timeout=120)
    return DRIVER


def _data(tmp_path, n=3000, p=6):
    X, y, _, _ = synth.generate(0, 0, n, p, 41)
    rng = np.random.default_rng(41)
    yl = X @ rng.normal(size=p) + rng.uniform(-1.0, 1.0, n)
    path = tmp_path / "data.bin"
    with open(path, "wb") as f:
        f.write(np.array([n, p], dtype=np.int64).tobytes())
        f.write(np.asfortranarray(X).tobytes(order="F"))
        f.write(np.ascontiguousarray(y).tobytes())
        f.write(np.ascontiguousarray(yl).tobytes())
    return X, y, yl, str(path)


def _run(mode, path):
    out = subprocess.run([_driver(), mode, path], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.splitlines()
    assert lines[-1] == "ok", out.stdout
    i, j = lines.index("summary_begin"), lines.index("summary_end")
    kv = {}
    for ln in lines[:i] + lines[j + 1:-1]:
        k, *v = ln.split()
        kv[k] = v
    return kv, "\n".join(lines[i + 1:j])


def _f(v):
    return np.array([float(x) for x in v])


def test_c_driver_lm_over_external_partials_and_errors(tmp_path):
    X, _, yl, path = _data(tmp_path)
    kv, summary = _run("cpu", path)
    # requires -> SGLM_EINVAL (1) before any device work
    assert kv["create_null_devs"] == ["1"] and kv["create_zero_devs"] == ["1"]
    if "create_no_device" in kv:  # no GPU: SGLM_EHIP (3), no handle -- loudly, no CPU fallback
        assert kv["create_no_device"] == ["3", "1"]
    assert kv["abi"] == ["8"]
    # two partitions on two threads, one in-process all-reduce: both ranks hold the same fit, bit for bit
    assert kv["ranks_bitwise"] == ["1"] and kv["lm_npart"] == ["2"]
    r = po.fit_lm(X, yl, npart=2)
    assert rel(_f(kv["lm_coefs"]), r["coefs"]) < 1e-9 and rel(_f(kv["lm_stderr"]), r["stderr"]) < 1e-9
    st = _f(kv["lm_stats"])
    assert rel(st[:4], [r["sse"], r["r2"], r["fstat"], r["sigma"]]) < 1e-9 and st[4] == len(yl)
    assert "Multiple R-Squared" in summary and all(f"x{j}" in summary for j in range(X.shape[1]))


@pytest.mark.gpu
def test_c_driver_fits_on_the_device(tmp_path):
    X, y, yl, path = _data(tmp_path, n=20_000, p=8)
    kv, summary = _run("gpu", path)
    assert kv["set_data_bad_n"] == ["1"]  # require(n >= 1) -> SGLM_EINVAL
    o = po.fit_glm(X, y)
    assert int(kv["glm_iter"][0]) == o.iter
    assert rel(_f(kv["glm_coefs"]), o.coefs) < 1e-9 and rel(_f(kv["glm_stderr"]), o.stderr) < 1e-9
    gs = _f(kv["glm_stats"])
    assert rel(gs[:4], [o.deviance, o.null_deviance, o.pearson, o.loglik]) < 1e-9 and gs[4] == len(y)
    mu = 1.0 / (1.0 + np.exp(-(X[:5] @ _f(kv["glm_coefs"]))))
    assert rel(_f(kv["mu_head"]), mu) < 1e-13
    assert f"Number of Fisher Scoring iterations: {o.iter}" in summary
    r = po.fit_lm(X, yl)
    assert rel(_f(kv["lm_coefs"]), r["coefs"]) < 1e-9 and rel(_f(kv["lm_stderr"]), r["stderr"]) < 1e-9
    assert rel(_f(kv["lm_stats"])[:4], [r["sse"], r["r2"], r["fstat"], r["sigma"]]) < 1e-9
    assert kv["kernel"][0].startswith("irls_narrow_kernel<1,")
