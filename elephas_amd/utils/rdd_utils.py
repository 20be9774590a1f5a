"""numpy <-> RDD adapters (reference elephas/utils/rdd_utils.py:10-85)."""
from typing import Optional, Tuple

import numpy as np

from ..data.linalg import LabeledPoint
from ..mllib.adapter import from_vector, to_vector


def to_simple_rdd(sc, features: np.ndarray, labels: np.ndarray):
    """numpy features/labels -> RDD of (x, y) pairs (``parallelize``: contiguous slices).

    The partitions are columnar views of the two arrays (data/rdd.py ColumnarPartition):
    they iterate as (x, y) pairs like the reference's, but the training path uploads
    the arrays directly instead of rebuilding them row by row."""
    from ..data.rdd import RDD
    features, labels = np.asarray(features), np.asarray(labels)
    return RDD.from_arrays(features, labels, sc.defaultParallelism, sc)


def to_labeled_point(sc, features: np.ndarray, labels: np.ndarray, categorical: bool = False):
    labeled_points = [LabeledPoint(np.argmax(y) if categorical else y, to_vector(x))
                      for x, y in zip(features, labels)]
    return sc.parallelize(labeled_points)


def from_labeled_point(rdd, categorical: bool = False, nb_classes: Optional[int] = None) -> Tuple[np.ndarray, np.ndarray]:
    features_and_labels = rdd.map(lambda lp: (from_vector(lp.features), int(lp.label)))
    features, labels = zip(*features_and_labels.collect())
    features = np.array(features)
    labels = np.array(labels)
    if categorical:
        if not nb_classes:
            nb_classes = np.max(labels) + 1
        labels = np.stack([encode_label(x, nb_classes) for x in labels])
    return features, labels


def encode_label(label, nb_classes: int) -> np.ndarray:
    encoded = np.zeros(nb_classes)
    encoded[int(label)] = 1.0
    return encoded


def lp_to_simple_rdd(lp_rdd, categorical: bool = False, nb_classes: int = None):
    if categorical:
        if not nb_classes:
            nb_classes = lp_rdd.map(lambda lp: lp.label).map(int).max() + 1
        return lp_rdd.map(lambda lp: (from_vector(lp.features), encode_label(lp.label, nb_classes)))
    return lp_rdd.map(lambda lp: (from_vector(lp.features), lp.label))
