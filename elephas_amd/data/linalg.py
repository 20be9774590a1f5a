"""MLlib/ML linear-algebra value types (pyspark.mllib.linalg / pyspark.ml.linalg
subset used by the reference adapters: reference elephas/mllib/adapter.py:1-35,
utils/rdd_utils.py:23-85, ml/adapter.py:11-46).

``DenseMatrix`` stores values COLUMN-major like Spark.  ``to_matrix`` in the
adapter keeps the reference's behaviour of handing it a row-major ``ravel()``
 unless asked to transpose correctly.
"""
from __future__ import annotations

from typing import Iterable, Sequence

import numpy as np


class Vector:
    def toArray(self) -> np.ndarray:
        raise NotImplementedError


class DenseVector(Vector):
    __slots__ = ("array",)

    def __init__(self, ar):
        self.array = np.asarray(ar, dtype=np.float64).reshape(-1)

    def toArray(self) -> np.ndarray:
        return self.array

    def __getattr__(self, item):
        # pyspark's DenseVector delegates unknown attributes (shape, ...) to the array
        if item == "array" or item.startswith("__"):
            raise AttributeError(item)
        return getattr(self.array, item)

    @property
    def values(self):
        return self.array

    @property
    def size(self):
        return self.array.size

    def __len__(self):
        return self.array.size

    def __getitem__(self, i):
        return self.array[i]

    def __iter__(self):
        return iter(self.array)

    def dot(self, other):
        o = other.toArray() if isinstance(other, Vector) else np.asarray(other)
        return float(np.dot(self.array, o))

    def norm(self, p):
        return float(np.linalg.norm(self.array, p))

    def __eq__(self, other):
        if isinstance(other, Vector):
            return np.array_equal(self.toArray(), other.toArray())
        return False

    def __hash__(self):
        return hash(self.array.tobytes())

    def __repr__(self):
        return "DenseVector([" + ", ".join(f"{v:g}" for v in self.array[:20]) + (", ..." if self.size > 20 else "") + "])"

    def __reduce__(self):
        return (DenseVector, (self.array.tolist(),))


class SparseVector(Vector):
    def __init__(self, size, indices, values=None):
        self.size = int(size)
        if values is None:  # dict form
            items = sorted(dict(indices).items())
            indices = [k for k, _ in items]
            values = [v for _, v in items]
        self.indices = np.asarray(indices, dtype=np.int32)
        self.values = np.asarray(values, dtype=np.float64)

    def toArray(self):
        a = np.zeros(self.size)
        a[self.indices] = self.values
        return a

    def __len__(self):
        return self.size

    def __repr__(self):
        return f"SparseVector({self.size}, {dict(zip(self.indices.tolist(), self.values.tolist()))})"


class Vectors:
    @staticmethod
    def dense(*elements):
        if len(elements) == 1 and not isinstance(elements[0], (int, float)):
            return DenseVector(elements[0])
        return DenseVector(elements)

    @staticmethod
    def sparse(size, *args):
        return SparseVector(size, *args)

    @staticmethod
    def fromML(vec):
        return vec

    @staticmethod
    def asML(vec):
        return vec


class Matrix:
    def toArray(self) -> np.ndarray:
        raise NotImplementedError


class DenseMatrix(Matrix):
    def __init__(self, numRows, numCols, values, isTransposed=False):
        self.numRows, self.numCols = int(numRows), int(numCols)
        self.values = np.asarray(values, dtype=np.float64).reshape(-1)
        if self.values.size != self.numRows * self.numCols:
            raise ValueError("values size does not match the matrix shape")
        self.isTransposed = isTransposed

    def toArray(self) -> np.ndarray:
        if self.isTransposed:
            return self.values.reshape(self.numRows, self.numCols)
        return self.values.reshape(self.numCols, self.numRows).T.copy()

    def __repr__(self):
        return f"DenseMatrix({self.numRows}, {self.numCols}, ...)"


class Matrices:
    @staticmethod
    def dense(numRows, numCols, values):
        return DenseMatrix(numRows, numCols, values)


class LabeledPoint:
    __slots__ = ("label", "features")

    def __init__(self, label, features):
        lab = np.asarray(label, dtype=np.float64)
        if lab.size != 1:   # pyspark: float(label) -- a multi-element label is an error
            raise TypeError(f"LabeledPoint label must be a scalar, got shape {lab.shape}")
        self.label = float(lab.reshape(-1)[0])
        self.features = features if isinstance(features, Vector) else DenseVector(features)

    def __repr__(self):
        return f"LabeledPoint({self.label}, {self.features!r})"

    def __reduce__(self):
        return (LabeledPoint, (self.label, self.features))
