"""A minimal columnar stand-in for the Spark DataFrames the reference API takes.

The reference's fit entry points receive Spark SQL DataFrames (GLM.scala:597-995,
LM.scala:241) and only ever use: column names (`columns`), column types (`dtypes`,
all must be DoubleType), row counts (`count`) and the partition count
(`rdd.partitions.size`), which selects the single- or multi-partition driver.  `Frame`
keeps exactly that surface over numpy columns.
"""
from __future__ import annotations

import json
from typing import Dict, Iterable, List, Sequence

import numpy as np


class _RDD:
    class _Parts:
        def __init__(self, n):
            self._n = n

        def size(self):
            return self._n

    def __init__(self, npart):
        self.partitions = _RDD._Parts(npart)


class Frame:
    def __init__(self, data: Dict[str, Sequence], npartitions: int = 1, columns: Iterable[str] = None):
        cols = list(columns) if columns is not None else list(data.keys())
        self._data = {}
        for c in cols:
            v = np.asarray(data[c])
            if v.dtype.kind in "iub":
                v = v.astype(np.float64) if v.dtype.kind == "b" else v
            self._data[c] = v
        n = {len(v) for v in self._data.values()}
        if len(n) > 1:
            raise ValueError("columns differ in length")
        self._n = n.pop() if n else 0
        self.npartitions = int(npartitions)
        self.rdd = _RDD(self.npartitions)

    # ---- the surface the reference uses ----
    @property
    def columns(self) -> List[str]:
        return list(self._data.keys())

    @property
    def dtypes(self):
        def t(v):
            if v.dtype == np.float64:
                return "DoubleType"
            if v.dtype.kind in "iu":
                return "LongType"
            if v.dtype.kind in "OUS":
                return "StringType"
            return str(v.dtype)
        return [(c, t(v)) for c, v in self._data.items()]

    def count(self) -> int:
        return self._n

    # ---- helpers ----
    def __getitem__(self, c):
        return self._data[c]

    def select(self, *cols) -> "Frame":
        cols = cols[0] if len(cols) == 1 and not isinstance(cols[0], str) else cols
        return Frame({c: self._data[c] for c in cols}, self.npartitions)

    def repartition(self, npartitions: int) -> "Frame":
        return Frame(dict(self._data), npartitions)

    def coalesce(self, npartitions: int) -> "Frame":
        return Frame(dict(self._data), min(npartitions, self.npartitions))

    def with_column(self, name: str, values) -> "Frame":
        d = dict(self._data)
        d[name] = np.asarray(values)
        return Frame(d, self.npartitions)

    def to_matrix(self) -> np.ndarray:
        """Column-major n x p float64 matrix (Breeze DenseMatrix layout)."""
        if not self._data:
            return np.zeros((self._n, 0), order="F")
        return np.asfortranarray(np.column_stack([np.asarray(v, dtype=np.float64) for v in self._data.values()]))

    def to_vector(self) -> np.ndarray:
        if len(self._data) != 1:
            raise ValueError("expected a single column")
        return np.asarray(next(iter(self._data.values())), dtype=np.float64)

    @staticmethod
    def from_pandas(df, npartitions: int = 1) -> "Frame":
        return Frame({c: df[c].to_numpy() for c in df.columns}, npartitions)

    @staticmethod
    def read_json(path: str, npartitions: int = 1) -> "Frame":
        """Spark's read.json schema: union of keys, sorted by name; integral values -> Long."""
        rows = [json.loads(l) for l in open(path) if l.strip()]
        keys = sorted({k for r in rows for k in r})
        data = {}
        for k in keys:
            vals = [r.get(k) for r in rows]
            if all(isinstance(v, float) or isinstance(v, int) for v in vals):
                data[k] = np.array(vals, dtype=np.float64 if any(isinstance(v, float) for v in vals) else np.int64)
            else:
                data[k] = np.array(vals, dtype=object)
        return Frame(data, npartitions)

    def __repr__(self):
        return f"Frame({self._n} rows, {self.columns}, npartitions={self.npartitions})"
