"""``pyspark.mllib.linalg`` (dense matrices are column-major, as in Spark)."""
from ...data.linalg import DenseMatrix, DenseVector, Matrices, Matrix, SparseVector, Vector, Vectors  # noqa: F401
