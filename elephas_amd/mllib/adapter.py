"""numpy <-> MLlib linalg (reference elephas/mllib/adapter.py:1-35).

``to_matrix`` reproduces the reference exactly: it hands a row-major
``ravel()`` to the column-major ``Matrices.dense``, so
``from_matrix(to_matrix(a))`` is ``a`` only for symmetric layouts; pass
``column_major=True`` for the corrected transfer."""
import numpy as np

from ..data.linalg import Matrices, Matrix, Vector, Vectors


def from_matrix(matrix: Matrix) -> np.ndarray:
    return matrix.toArray()


def to_matrix(np_array: np.ndarray, column_major: bool = False) -> Matrix:
    if len(np_array.shape) == 2:
        vals = np_array.T.ravel() if column_major else np_array.ravel()
        return Matrices.dense(np_array.shape[0], np_array.shape[1], vals)
    raise Exception("An MLLib Matrix can only be created from a two-dimensional " +
                    "numpy array, got {}".format(len(np_array.shape)))


def from_vector(vector: Vector) -> np.ndarray:
    return vector.toArray()


def to_vector(np_array: np.ndarray) -> Vector:
    if len(np_array.shape) == 1:
        return Vectors.dense(np_array)
    raise Exception("An MLLib Vector can only be created from a one-dimensional " +
                    "numpy array, got {}".format(len(np_array.shape)))
