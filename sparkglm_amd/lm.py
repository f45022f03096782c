"""`LM` -- the reference's Scala linear-model API, over the MI355X engine.

Mirrors com.Alteryx.sparkGLM.LM (LM.scala): `LM.fit(x, y)` with its `require` checks,
the `LM` model class with `predict` and `summary`, and `SummaryLM`.  The normal-equation
work (rowPartitionedComponents, inv, rowPartitionedSSE) runs in the engine
(sglm_fit_lm); the printed summary comes from sglm_lm_summary.

As in the reference, no intercept is added (supply an `intercept` column) and
r2 = SSR/SST (LM.scala:185), which exceeds 1 without an intercept.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import List

import numpy as np

from . import _lib as L
from .frame import Frame
from .glm import _engine, _require


@dataclass
class PreLM:
    """LM.scala:10-14"""
    coefs: np.ndarray
    xtxi: np.ndarray
    sse: float
    r2: float
    fStat: float


class LMModel:
    """class LM (LM.scala:16-64)."""

    def __init__(self, xnames, yname, coefs, stdErr, sigma, r2, fStat, nrow, npart):
        self.xnames: List[str] = list(xnames)
        self.yname: str = yname
        self.coefs = coefs
        self.stdErr: List[float] = list(stdErr)
        self.sigma = sigma
        self.r2 = r2
        self.fStat = fStat
        self.nrow = nrow
        self.npart = npart

    def predict(self, newData: Frame, device: int = 0) -> Frame:
        """LM.scala:29-61: (index, value) rows of newX * coefs, on the GPU (sglm_predict_new: the
        new rows stream through a scratch buffer; a design resident on the device stays put).

        As the reference, newX is newData's whole matrix in its own column order (LM.scala:40,
        54: dfToDenseMatrix / dataFrameToMatrix of newData), so a frame with extra columns fails
        Breeze's dimension check.  With ``glm.strict = False`` the model's columns are selected
        by name instead (extension)."""
        from . import glm as _glm
        _require(len(set(self.xnames) - set(newData.columns)) == 0,
                 "Not all predictors in the estimation data are in the data to be predicted")
        if _glm.strict:
            newX = newData.to_matrix()
            if newX.shape[1] != len(self.xnames):
                raise L.IllegalArgumentException(f"requirement failed: Dimension mismatch: newData has "
                                                 f"{newX.shape[1]} columns, the model {len(self.xnames)} "
                                                 f"coefficients (breeze DenseMatrix *)")
        else:
            newX = newData.select(*self.xnames).to_matrix()
        vals = _engine(device).predict_new(newX, np.asarray(self.coefs, dtype=np.float64).reshape(-1))
        return Frame({"index": np.arange(len(vals), dtype=np.int64), "value": vals}, newData.npartitions)

    def summary(self) -> "SummaryLM":
        return SummaryLM(self)


class SummaryLM:
    """LM.scala:66-137"""

    def __init__(self, obj: LMModel):
        self.obj = obj
        self._lib = L.load()

    def _sd(self, x, d):
        return L.java_double_str(self._lib.sglm_sig_digits(float(x), d))

    def adjR2(self) -> float:
        o = self.obj
        return 1.0 - (((1.0 - o.r2) * (o.nrow - 1.0)) / (o.nrow - len(o.xnames) - 1.0))

    def dfm(self) -> float:
        return float(len(self.obj.xnames) - 1)

    def dfe(self) -> float:
        return float(int(self.obj.nrow) - len(self.obj.xnames))

    def coefficients(self):
        return list(np.asarray(self.obj.coefs).reshape(-1))

    def tVals(self):
        return [c / s for c, s in zip(self.coefficients(), self.obj.stdErr)]

    def pVals(self):
        return [self._lib.sglm_pval_t(t, self.dfe()) for t in self.tVals()]

    def formula(self) -> str:
        return self.obj.yname + " ~ " + " + ".join(self.obj.xnames)

    def coefsString(self) -> str:
        rows = ["%-12s %12s %12s %12s %12s" % ("", "Estimate", "Std. Error", "t value", "Pr(>|t|)")]
        for i, name in enumerate(self.obj.xnames):
            rows.append("%-12s %12s %12s %12s %12s" % (name, self._sd(self.coefficients()[i], 6),
                                                        self._sd(self.obj.stdErr[i], 6), self._sd(self.tVals()[i], 6),
                                                        self._sd(self.pVals()[i], 6)))
        return "\n".join(rows)

    def RSEString(self) -> str:
        return ("Residual standard error: " + self._sd(self.obj.sigma, 6) + " on " + L.java_double_str(self.dfe()) +
                " degrees of freedom")

    def R2String(self) -> str:
        rd = lambda x: L.java_double_str(self._lib.sglm_round_digits(float(x), 4))
        return "Multiple R-Squared: " + rd(self.obj.r2) + ", Adusted R-Squared: " + rd(self.adjR2())

    def FStatString(self) -> str:
        return ("F-statistic: " + self._sd(self.obj.fStat, 5) + " on " + L.java_double_str(self.dfm()) + " and " +
                L.java_double_str(self.dfe()) + " DF")

    def text(self) -> str:
        o = self.obj
        coefs = np.ascontiguousarray(np.asarray(o.coefs, dtype=np.float64).reshape(-1))
        se = np.ascontiguousarray(np.asarray(o.stdErr, dtype=np.float64))
        pre = L.PreLM(L.ptr(coefs), None, L.ptr(se), 0.0, o.r2, o.fStat, o.sigma, o.nrow, o.npart)
        names = (C.c_char_p * len(o.xnames))(*[n.encode() for n in o.xnames])
        need = self._lib.sglm_lm_summary(C.byref(pre), len(o.xnames), names, o.yname.encode(), None, 0)
        buf = C.create_string_buffer(int(need))
        self._lib.sglm_lm_summary(C.byref(pre), len(o.xnames), names, o.yname.encode(), buf, need)
        return buf.value.decode()

    def print(self) -> None:
        print(self.text(), end="")


class LM:
    """Namespace mirroring `object LM` (LM.scala:139-275)."""

    @staticmethod
    def fit(x: Frame, y: Frame, device: int = 0) -> LMModel:
        """LM.scala:241-274"""
        _require(all(t == "DoubleType" for _, t in x.dtypes), "The provided DataFrame must contain all 'DoubleType' columns")
        _require(x.rdd.partitions.size() == y.rdd.partitions.size(), "The two DataFrames must have the same number of paritions")
        _require(x.count() == y.count(), "The two DataFrames must have the same number of rows")
        _require(len(y.columns) == 1, "The 'y' DataFrame must have only one column")
        eng = _engine(device)
        eng.set_data(x.to_matrix(), y.to_vector())
        f = eng.fit_lm()
        return LMModel(x.columns, y.columns[0], f.coefs.reshape(-1, 1), list(f.stderr), f.sigma, f.r2, f.fstat,
                       float(y.count()), x.rdd.partitions.size())

    @staticmethod
    def fit_components(x: Frame, y: Frame, device: int = 0) -> PreLM:
        eng = _engine(device)
        eng.set_data(x.to_matrix(), y.to_vector())
        f = eng.fit_lm()
        return PreLM(f.coefs.reshape(-1, 1), f.xtxi, f.sse, f.r2, f.fstat)
