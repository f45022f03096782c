"""modelMatrix / matchCols, mirroring modelMatrix$Test.scala and utils$Test.scala
(the reference's dummyDF / oneLessCategoryDF / mixedDF fixtures, testData.scala:17-30)."""
import os

import numpy as np

from sparkglm_amd.frame import Frame
from sparkglm_amd.model_matrix import matchCols, modelMatrix

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def dummy_df():
    return Frame({"intField": np.array([1, 2, 3]), "strField": np.array(["a", "b", "c"], dtype=object),
                  "numField": np.array([1.0, 2.0, 3.0])})


def one_less_category_df():
    return Frame({"intField": np.array([1, 2, 3]), "strField": np.array(["a", "b", "a"], dtype=object),
                  "numField": np.array([1.0, 2.0, 3.0])})


def test_model_matrix_with_mixed_types():
    df = modelMatrix(dummy_df())
    assert len(df.columns) == 4
    assert all(c in df.columns for c in ["intField", "strField_b", "strField_c", "numField"])
    assert all(t == "DoubleType" for _, t in df.dtypes)
    # otherVars ++ dummies (modelMatrix.scala:26), when(field === level, 1).otherwise(0)
    assert df.columns == ["intField", "numField", "strField_b", "strField_c"]
    np.testing.assert_array_equal(df["strField_b"], [0.0, 1.0, 0.0])
    np.testing.assert_array_equal(df["strField_c"], [0.0, 0.0, 1.0])


def test_model_matrix_with_num_only():
    df = modelMatrix(dummy_df().select("numField", "intField"))
    assert df.columns == ["numField", "intField"]
    assert all(t == "DoubleType" for _, t in df.dtypes)


def test_model_matrix_with_str_only():
    df = modelMatrix(dummy_df().select("strField"))
    assert df.columns == ["strField_b", "strField_c"]
    assert all(t == "DoubleType" for _, t in df.dtypes)


def test_model_matrix_linear_reg_data():
    raw = Frame.read_json(os.path.join(GOLD, "linear_reg_mixed.json"))
    raw = raw.select("intercept", "x1", "x2", "x3", "x4", "x5", "x6", "x7", "y")
    df = modelMatrix(raw)
    assert len(df.columns) == 10
    assert all(c in df.columns for c in ["intercept", "x1", "x2", "x3", "x4", "x5", "x6", "x7_b", "x7_c", "y"])
    assert all(t == "DoubleType" for _, t in df.dtypes)
    x7 = raw["x7"]
    np.testing.assert_array_equal(df["x7_b"], (x7 == "b").astype(float))
    np.testing.assert_array_equal(df["x7_c"], (x7 == "c").astype(float))


def test_match_cols():
    df = modelMatrix(dummy_df())
    missing = modelMatrix(one_less_category_df())
    out = matchCols(df, missing)
    assert len(out.columns) == 4
    assert all(t == "DoubleType" for _, t in out.dtypes)
    assert all(c in out.columns for c in ["intField", "strField_b", "strField_c", "numField"])
    assert out.columns[0] == "strField_c"  # missing columns first (utils.scala:23-26)
    assert set(out["strField_c"].tolist()) == {0.0}
    out2 = matchCols(df.columns, missing)
    assert out2.columns == out.columns
