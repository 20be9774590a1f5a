"""numpy <-> DataFrame adapters (reference elephas/ml/adapter.py:1-47)."""
from typing import Optional

import numpy as np

from ..data.linalg import LabeledPoint, Vector, Vectors
from ..data.sql import SparkSession
from ..utils.rdd_utils import from_labeled_point, lp_to_simple_rdd, to_labeled_point


def to_data_frame(sc, features: np.ndarray, labels: np.ndarray, categorical: bool = False):
    lp_rdd = to_labeled_point(sc, features, labels, categorical)
    return SparkSession.builder.getOrCreate().createDataFrame(lp_rdd)


def from_data_frame(df, categorical: bool = False, nb_classes: Optional[int] = None):
    lp_rdd = df.rdd.map(lambda row: LabeledPoint(row.label, row.features))
    return from_labeled_point(lp_rdd, categorical, nb_classes)


def df_to_simple_rdd(df, categorical: bool = False, nb_classes: Optional[int] = None,
                     features_col: str = "features", label_col: str = "label"):
    spark_session = SparkSession.builder.getOrCreate()
    df.createOrReplaceTempView("temp_table")
    selected_df = spark_session.sql(f"SELECT {features_col} AS features, {label_col} as label from temp_table")
    lp_rdd = selected_df.rdd.map(lambda row: LabeledPoint(row.label, Vectors.fromML(row.features)))
    nparts = df.rdd.getNumPartitions()
    if lp_rdd.getNumPartitions() != nparts:   # one worker per partition of the input DataFrame
        lp_rdd = lp_rdd.repartition(nparts)
    return lp_to_simple_rdd(lp_rdd, categorical, nb_classes)
