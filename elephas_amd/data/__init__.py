"""Spark-like host data layer (no JVM): SparkContext/RDD, DataFrame/SparkSession,
MLlib linalg, and the pyspark.ml pipeline pieces the Elephas API builds on."""
from .rdd import RDD, Broadcast, ColumnarPartition, SparkConf, SparkContext  # noqa: F401
from .linalg import DenseMatrix, DenseVector, LabeledPoint, Matrices, Matrix, SparseVector, Vector, Vectors  # noqa: F401
from .ml import Pipeline, PipelineModel  # noqa: F401
from .sql import (ArrayType, DataFrame, DoubleType, Row, SparkSession, StringType, StructField,  # noqa: F401
                  StructType, VectorUDT, col)
