"""Design-matrix preparation: modelMatrix dummy coding and matchCols (host side).

Mirrors the reference's DataFrame helpers that build the fitting inputs:

* ``modelMatrix(df)`` -- modelMatrix.scala:18-85.  String columns become k-1 binary
  columns named ``<field>_<level>`` (levels = the sorted distinct values minus the first,
  getLevels :53-55; ``when(field === level, 1).otherwise(0)``, explodeField :70-74), the
  other columns are kept in their order, the dummies are appended after them
  (``otherVars ++ createDummies``, :26-27), and every column is cast to DoubleType
  (castAll :78-84).  A DataFrame without string columns is only cast (:23-24).
* ``matchCols(est, score)`` / ``matchCols(xnames, score)`` -- utils.scala:21-33.  The
  columns of the estimation frame (or the name list) that the scoring frame lacks are
  prepended as 0.0 columns, followed by all of the scoring frame's columns.

The categorical columns are visited in their DataFrame order (the reference iterates a
Scala immutable Map keyed by Column, which keeps insertion order up to four keys).
This is one-off preprocessing before the data is uploaded: it runs
on the host, the result feeds ``Engine.set_data`` / ``GLM.fit`` / ``LM.fit`` unchanged.
"""
from __future__ import annotations

from typing import List, Sequence, Union

import numpy as np

from .frame import Frame


def _is_string(values) -> bool:
    v = np.asarray(values)
    return v.dtype.kind in "OUS"


def get_levels(df: Frame, field: str) -> List[str]:
    """getLevels (modelMatrix.scala:53-55): sorted distinct values, the first dropped."""
    vals = sorted({str(v) for v in df[field] if v is not None})
    return vals[1:]


def modelMatrix(df: Frame) -> Frame:
    """modelMatrix.scala:18-31."""
    cat = [c for c, t in df.dtypes if t == "StringType"]
    other = [c for c, t in df.dtypes if t != "StringType"]
    out = {c: np.asarray(df[c], dtype=np.float64) for c in other}
    for field in cat:
        col = df[field]
        for level in get_levels(df, field):
            name = f"{field}_{level}"
            out[name] = np.array([1.0 if (v is not None and str(v) == level) else 0.0 for v in col])
    return Frame(out, df.npartitions, columns=list(out.keys()))


def matchCols(est: Union[Frame, Sequence[str]], score: Frame) -> Frame:
    """utils.scala:21-33: missing estimation columns prepended to the scoring frame as 0.0."""
    names = est.columns if isinstance(est, Frame) else list(est)
    missing = [c for c in names if c not in score.columns]
    data = {c: np.zeros(score.count()) for c in missing}
    for c in score.columns:
        data[c] = score[c]
    return Frame(data, score.npartitions, columns=list(data.keys()))
