"""`GLM` -- the reference's Scala GLM API, over the MI355X engine.

Mirrors com.Alteryx.sparkGLM.GLM (GLM.scala): the sixteen `fit` overloads with their
`require` checks and defaults (tol = 1e-6, m = 1, offset = 0, verbose = false), the
PreGLM / GLM result objects, `createObj` and `summary`.  The fit driver bodies
(fitSingleBinomial / fitMultipleBinomial) are replaced by the engine (sglm_fit_glm).

Faithful-to-the-reference behaviour (``strict = True``, the default):
  * any family string fits binomial unless it names an extension family; binomial links
    are "logit", "probit" and anything else = cloglog (GLM.scala:264-299);
  * only the 4-argument overload runs on a multi-partition DataFrame; every other
    overload requires a single partition ("The DataFrame must be in a single partition",
    utils.scala:43-44) because the reference routes them to fitSingle;
  * fit(y, x, offset, family, link, tol, m) ignores the offset (GLM.scala:789-792);
  * the first iteration uses mu = mean(y) on one partition, unlink(link(mean(y))) on
    several (GLM.scala:263 vs 370-371); npart reports the partition count.
With ``strict = False`` every overload runs on partitioned data and honours its offset.
The extension families "gaussian", "poisson" and "gamma" (canonical links; prior weights
through `fit_weighted`) follow R's family objects on the same IRLS skeleton.  Their `loglik`
is R's logLik; `aic` stays createObj's -2 loglik + 2p (GLM.scala:70), which counts the
coefficients only -- R's AIC(glm) for gaussian and Gamma adds 2 for the dispersion parameter,
so it is 2 higher than `aic` here for those two families.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from . import _lib as L
from .engine import Engine
from .frame import Frame

strict = True
_engines = {}


def _engine(device: int = 0) -> Engine:
    e = _engines.get(device)
    if e is None:
        e = _engines[device] = Engine(device)
    return e


def _require(cond: bool, msg: str):
    if not cond:
        raise L.IllegalArgumentException("requirement failed: " + msg)


@dataclass
class PreGLM:
    """GLM.scala:25-33"""
    coefs: np.ndarray
    stdErr: List[float]
    deviance: float
    nullDeviance: float
    pearson: float
    loglik: float
    iter: int
    nrow: float
    npart: int


@dataclass
class GLMModel:
    """The GLM case class (GLM.scala:35-51)."""
    xnames: List[str]
    yname: str
    coefs: np.ndarray
    stdErr: List[float]
    dfResidual: float
    dfNull: float
    deviance: float
    nullDeviance: float
    pDispersion: float
    pearson: float
    loglik: float
    family: str
    link: str
    aic: float
    iter: int
    nrow: float
    npart: int

    def predict(self, newData: Frame, type: str = "response", offset: Optional[Frame] = None,
                m: Optional[Frame] = None, device: int = 0) -> Frame:
        """Extension (the reference has no GLM predict): (index, value) rows of the
        linear predictor newX * coefs (+ offset) on the "link" scale, or of mu = unlink(eta, m)
        on the "response" scale (m = binomial trials, default 1) -- R's predict.glm(type=).
        Runs on the GPU through sglm_predict_new; newData's columns are taken by the model's
        names."""
        _require(len(set(self.xnames) - set(newData.columns)) == 0,
                 "Not all predictors in the estimation data are in the data to be predicted")
        fam, lnk = _engine_family_link(self.family, self.link)
        newX = newData.select(*self.xnames).to_matrix()
        vals = _engine(device).predict_new(newX, np.asarray(self.coefs, dtype=np.float64).reshape(-1), fam, lnk,
                                           type, None if offset is None else offset.to_vector(),
                                           None if m is None else m.to_vector())
        return Frame({"index": np.arange(len(vals), dtype=np.int64), "value": vals}, newData.npartitions)


def _engine_family_link(family: str, link: str):
    f = family.lower()
    if f in ("gaussian", "poisson", "gamma"):
        canon = L.CANONICAL_LINK[f]
        _require(link == canon, f"family {family} supports only the {canon} link")
        return f, canon
    # binomial, including any unrecognised family string (GLM.scala:486-590)
    if link == "logit":
        return "binomial", "logit"
    if link == "probit":
        return "binomial", "probit"
    return "binomial", "cloglog"


def _check_inputs(y: Frame, x: Frame):
    # GLM.scala:602-609 (identical in every overload)
    _require(all(t == "DoubleType" for _, t in x.dtypes), "The provided DataFrame must contain all 'DoubleType' columns")
    _require(x.rdd.partitions.size() == y.rdd.partitions.size(), "The two DataFrames must have the same number of paritions")
    _require(x.count() == y.count(), "The two DataFrames must have the same number of rows")
    _require(len(y.columns) == 1, "The 'y' DataFrame must have only one column")


def _single_partition(df: Frame):
    # utils.dfToDenseMatrix (utils.scala:43-46)
    _require(df.rdd.partitions.size() == 1, "The DataFrame must be in a single partition")
    _require(all(t == "DoubleType" for _, t in df.dtypes), "The provided DataFrame must contain all 'DoubleType' columns")


def _to_pre(f) -> PreGLM:
    return PreGLM(f.coefs.reshape(-1, 1), list(f.stderr), f.deviance, f.null_deviance, f.pearson, f.loglik, f.iter,
                  f.nrow, f.npart)


def _fit_components(y: Frame, x: Frame, family: str, link: str, tol: float, verbose: bool,
                    offset: Optional[Frame] = None, m: Optional[Frame] = None, prior: Optional[Frame] = None,
                    device: int = 0) -> PreGLM:
    npart = x.rdd.partitions.size()
    fam, lnk = _engine_family_link(family, link)
    for extra in (offset, m, prior):
        if extra is not None:
            if strict or npart == 1:
                _single_partition(extra)
            _require(extra.count() == y.count(), "The two DataFrames must have the same number of rows")
    eng = _engine(device)
    eng.set_data(x.to_matrix(), y.to_vector(), None if m is None else m.to_vector(),
                 None if offset is None else offset.to_vector(), None if prior is None else prior.to_vector())
    f = eng.fit_glm(fam, lnk, tol=tol, verbose=verbose, init="single" if npart == 1 else "multiple", npart=npart)
    return _to_pre(f)


def _pre_struct(pre: PreGLM):
    coefs = np.ascontiguousarray(np.asarray(pre.coefs, dtype=np.float64).reshape(-1))
    se = np.ascontiguousarray(np.asarray(pre.stdErr, dtype=np.float64))
    s = L.PreGLM(L.ptr(coefs), L.ptr(se), pre.deviance, pre.nullDeviance, pre.pearson, pre.loglik, pre.iter,
                 pre.nrow, pre.npart, None, 0)
    return s, (coefs, se)


class GLM:
    """Namespace mirroring `object GLM` (GLM.scala:55-1026)."""

    @staticmethod
    def createObj(x: Frame, y: Frame, pre: PreGLM, family: str, link: str) -> GLMModel:
        """GLM.scala:59-88 (derived fields computed by sglm_glm_create_obj)."""
        lib = L.load()
        s, keep = _pre_struct(pre)
        s.nrow = float(y.count())
        d = L.GlmDerived()
        L.check(lib.sglm_glm_create_obj(C.byref(s), len(pre.stdErr), C.byref(d)))
        return GLMModel(x.columns, y.columns[0], pre.coefs, pre.stdErr, d.df_residual, d.df_null, pre.deviance,
                        pre.nullDeviance, d.p_dispersion, pre.pearson, pre.loglik, family, link, d.aic, pre.iter,
                        pre.nrow, pre.npart)

    @staticmethod
    def fit(y: Frame, x: Frame, *args, device: int = 0) -> GLMModel:
        """The sixteen Scala overloads (GLM.scala:597-995), dispatched on argument types."""
        args = list(args)
        offset = None
        if args and isinstance(args[0], Frame):
            offset = args.pop(0)
        _require(len(args) >= 2 and isinstance(args[0], str) and isinstance(args[1], str),
                 "fit(y, x, [offset,] family, link, ...)")
        family, link = args[0], args[1]
        tol, m, verbose = 1e-6, None, False
        rest = args[2:]
        kinds = []
        for a in rest:
            if isinstance(a, bool):
                verbose = a
                kinds.append("verbose")
            elif isinstance(a, (float, int)):
                tol = float(a)
                kinds.append("tol")
            elif isinstance(a, Frame):
                m = a
                kinds.append("m")
            else:
                raise TypeError(f"unsupported overload argument {a!r}")
        _require(kinds in ([], ["m"], ["tol"], ["tol", "m"], ["verbose"], ["m", "verbose"], ["tol", "verbose"],
                           ["tol", "m", "verbose"]), "no GLM.fit overload matches the arguments")
        _check_inputs(y, x)
        npart = x.rdd.partitions.size()
        four_arg = offset is None and not kinds
        if strict:
            if offset is not None and kinds == ["tol", "m"]:
                offset = None  # GLM.scala:789-792: this overload calls fitSingle without the offset
            if npart > 1 and not four_arg:
                # "Will change to fitDouble": fitSingle -> dfToDenseMatrix requires one partition
                _single_partition(x)
        pre = _fit_components(y, x, family, link, tol, verbose, offset=offset, m=m, device=device)
        return GLM.createObj(x, y, pre, family, link)

    @staticmethod
    def fit_weighted(y: Frame, x: Frame, family: str, link: str, prior: Frame, offset: Frame = None,
                     m: Frame = None, tol: float = 1e-6, verbose: bool = False, device: int = 0) -> GLMModel:
        """Extension: prior weights (R's `weights=`), on any partitioning."""
        _check_inputs(y, x)
        global strict
        saved, strict = strict, False
        try:
            pre = _fit_components(y, x, family, link, tol, verbose, offset=offset, m=m, prior=prior, device=device)
        finally:
            strict = saved
        return GLM.createObj(x, y, pre, family, link)

    @staticmethod
    def summary_string(obj: GLMModel) -> str:
        lib = L.load()
        pre = PreGLM(obj.coefs, obj.stdErr, obj.deviance, obj.nullDeviance, obj.pearson, obj.loglik, obj.iter,
                     obj.nrow, obj.npart)
        s, keep = _pre_struct(pre)
        names = (C.c_char_p * len(obj.xnames))(*[n.encode() for n in obj.xnames])
        need = lib.sglm_glm_summary(C.byref(s), len(obj.xnames), names, obj.yname.encode(), obj.family.encode(),
                                    obj.link.encode(), None, 0)
        buf = C.create_string_buffer(int(need))
        lib.sglm_glm_summary(C.byref(s), len(obj.xnames), names, obj.yname.encode(), obj.family.encode(),
                             obj.link.encode(), buf, need)
        return buf.value.decode()

    @staticmethod
    def summary(obj: GLMModel) -> None:
        """GLM.scala:998-1025 (prints)."""
        print(GLM.summary_string(obj), end="")
