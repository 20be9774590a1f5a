"""``pyspark.ml.linalg``."""
from ...data.linalg import DenseMatrix, DenseVector, Matrices, Matrix, SparseVector, Vector, Vectors  # noqa: F401
