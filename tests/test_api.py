"""The reference-mirroring host API (GLM.fit / LM.fit / model objects), read like the
reference's own ScalaTest/testthat suites.  The require(...) checks run on CPU; fits
need the GPU engine."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, iris_design, rel
from sparkglm_amd import IllegalArgumentException
from sparkglm_amd.frame import Frame
from sparkglm_amd.glm import GLM
from sparkglm_amd.lm import LM


def _frames(c, npart=1):
    X = c["X"]
    x = Frame({f"x{j}": X[:, j] for j in range(X.shape[1])}, npart)
    y = Frame({"y": c["y"]}, npart)
    return y, x


# ---------------------------------------------------------------- CPU: requirements
def test_require_double_columns():
    x = Frame({"a": np.array([1.0, 2.0]), "s": np.array(["u", "v"], dtype=object)})
    y = Frame({"y": np.array([0.0, 1.0])})
    with pytest.raises(IllegalArgumentException, match="must contain all 'DoubleType' columns"):
        GLM.fit(y, x, "binomial", "logit")
    with pytest.raises(IllegalArgumentException, match="must contain all 'DoubleType' columns"):
        LM.fit(x, y)


def test_require_partitions_rows_and_single_y():
    x = Frame({"a": np.arange(4.0)}, 2)
    with pytest.raises(IllegalArgumentException, match="same number of paritions"):
        GLM.fit(Frame({"y": np.arange(4.0)}, 1), x, "binomial", "logit")
    with pytest.raises(IllegalArgumentException, match="same number of rows"):
        LM.fit(Frame({"a": np.arange(4.0)}), Frame({"y": np.arange(3.0)}))
    with pytest.raises(IllegalArgumentException, match="only one column"):
        GLM.fit(Frame({"y": np.arange(4.0), "z": np.arange(4.0)}, 2), x, "binomial", "logit")


def test_offset_overloads_need_one_partition_like_the_reference(golden):
    # GLM.scala:638-642: "Will change to fitDouble" -> fitSingle -> dfToDenseMatrix require
    y, x = _frames(golden["logit"], npart=4)
    off = Frame({"o": np.zeros(len(golden["logit"]["y"]))}, 4)
    with pytest.raises(IllegalArgumentException, match="must be in a single partition"):
        GLM.fit(y, x, off, "binomial", "logit")
    with pytest.raises(IllegalArgumentException, match="must be in a single partition"):
        GLM.fit(y, x, "binomial", "logit", 1e-8)


def test_frame_read_json_schema():
    f = Frame.read_json(os.path.join(GOLDEN, "linear_reg_mixed.json"))
    assert f.columns == sorted(f.columns)  # Spark's JSON schema inference orders fields by name
    d = dict(f.dtypes)
    assert d["x7"] == "StringType" and d["rec_id"] == "StringType" and d["y"] == "DoubleType"
    assert f.count() == 1000


# ---------------------------------------------------------------- GPU: fits
@pytest.mark.gpu
def test_glm_fit_four_arg_single_and_partitioned(golden):
    c = golden["logit"]
    y, x = _frames(c)
    g = GLM.fit(y, x, "binomial", "logit")
    assert g.iter == int(c["scalars"][4]) and g.npart == 1
    assert rel(np.ravel(g.coefs), c["coefs"]) < 1e-9 and rel(g.stdErr, c["stderr"]) < 1e-9
    assert g.xnames == x.columns and g.yname == "y" and g.family == "binomial" and g.link == "logit"
    p, n = len(g.xnames), len(c["y"])
    assert g.dfResidual == n - p and g.dfNull == n - 1
    assert g.aic == -2 * g.loglik + 2 * p and rel(g.pDispersion, g.pearson / (n - p)) < 1e-15
    c4 = golden["logit_npart4"]
    y4, x4 = _frames(c4, npart=4)
    g4 = GLM.fit(y4, x4, "Binomial", "logit")
    assert g4.npart == 4 and g4.iter == int(c4["scalars"][4])
    assert rel(np.ravel(g4.coefs), c4["coefs"]) < 1e-9


@pytest.mark.gpu
def test_glm_overloads_with_offset_and_m(golden):
    c = golden["binomial_m_offset"]
    y, x = _frames(c)
    off, m = Frame({"o": c["offset"]}), Frame({"m": c["m"]})
    full = GLM.fit(y, x, off, "binomial", "logit", m)
    assert rel(np.ravel(full.coefs), c["coefs"]) < 1e-9 and full.iter == int(c["scalars"][4])
    same = GLM.fit(y, x, off, "binomial", "logit", 1e-6, m, False)
    np.testing.assert_array_equal(np.ravel(same.coefs), np.ravel(full.coefs))
    # GLM.scala:789-792: this overload drops the offset
    dropped = GLM.fit(y, x, off, "binomial", "logit", 1e-6, m)
    no_off = GLM.fit(y, x, "binomial", "logit", 1e-6, m)
    np.testing.assert_array_equal(np.ravel(dropped.coefs), np.ravel(no_off.coefs))
    # unknown link -> cloglog, unknown family -> binomial (GLM.scala:264-270, 486-490)
    yb, xb = _frames(golden["cloglog"])
    a = GLM.fit(yb, xb, "whatever", "complementary")
    assert rel(np.ravel(a.coefs), golden["cloglog"]["coefs"]) < 1e-9


@pytest.mark.gpu
def test_glm_summary_text(golden):
    y, x = _frames(golden["logit"])
    g = GLM.fit(y, x, "binomial", "logit")
    t = GLM.summary_string(g)
    lines = t.split("\n")
    assert lines[0] == "Model:" and lines[1] == "y ~ x0 + x1 + x2 + x3 + x4"
    assert lines[2] == "Family: binomial" and lines[3] == "Link: logit"
    assert "%-12s %12s %12s %12s %12s" % ("", "Estimate", "Std. Error", "z value", "Pr(>|z|)") in t
    assert f"Number of Fisher Scoring iterations: {g.iter}" in t
    assert "on 599 degress of freedom" in t and "on 595 degress of freedom" in t


@pytest.mark.gpu
def test_lm_iris_like_the_r_tests(iris):
    # R/pkg/tests/testthat/test_LM.R:26-45
    X, yv, names = iris_design(iris)
    x = Frame({nm: X[:, j] for j, nm in enumerate(names)})
    y = Frame({"Sepal_Width": yv})
    model = LM.fit(x, y)
    assert model.xnames == names
    s = model.summary()
    assert s.formula() == "Sepal_Width ~ Petal_Length + Petal_Width + Species_versicolor + Species_virginica"
    assert s.R2String() == "Multiple R-Squared: 3.8443, Adusted R-Squared: 3.9228"
    assert s.R2String() in s.text() and s.RSEString() in s.text() and s.FStatString() in s.text()
    pred = model.predict(x)
    assert pred.count() == 150 and pred.columns == ["index", "value"]
    assert rel(pred["value"], X @ np.ravel(model.coefs)) < 1e-13


@pytest.mark.gpu
def test_lm_predict_test_rdd_single_and_multi_partition():
    # lmPredict$Test.scala:11-35
    d = np.loadtxt(os.path.join(GOLDEN, "test_rdd.csv"), delimiter=",", skiprows=1)
    for npart in (1, 4):
        x = Frame({"intercept": d[:, 0], "x": d[:, 1]}, npart)
        y = Frame({"y": d[:, 2]}, npart)
        m = LM.fit(x, y)
        pred = m.predict(x)
        assert pred.npartitions == npart and len(pred.columns) == 2 and pred["index"].max() == 49
