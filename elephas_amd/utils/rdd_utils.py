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
    """numpy features/labels -> RDD of LabeledPoints (labels: class index when
    ``categorical``). Partitions are columnar (data/rdd.py LabeledPointPartition): they
    iterate as LabeledPoint objects, and lp_to_simple_rdd converts them as arrays."""
    from ..data.rdd import LabeledPointPartition, RDD
    features, labels = np.asarray(features), np.asarray(labels)
    scalar_labels = labels.ndim == 1 or (labels.ndim == 2 and labels.shape[1] == 1)
    if features.ndim != 2 or len(features) != len(labels) or (not categorical and not scalar_labels):
        # anything not a row matrix (or multi-column labels without ``categorical``) keeps
        # the reference's per-row construction, and its errors
        return sc.parallelize([LabeledPoint(np.argmax(y) if categorical else y, to_vector(x))
                               for x, y in zip(features, labels)])
    lab = np.argmax(labels.reshape(len(labels), -1), axis=1) if categorical else labels.reshape(len(labels), -1)[:, 0]
    lab = lab.astype(np.float64)
    n, k = len(features), max(1, sc.defaultParallelism)
    return RDD([LabeledPointPartition(features[i * n // k:(i + 1) * n // k], lab[i * n // k:(i + 1) * n // k])
                for i in range(k)], sc)


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
    from ..data.rdd import ColumnarPartition, LabeledPointPartition, RDD
    parts = lp_rdd.partitions() if hasattr(lp_rdd, "partitions") else None
    if parts and all(isinstance(p, LabeledPointPartition) for p in parts):
        # columnar LabeledPoints: the same (features, label) pairs as the per-row path,
        # built as arrays; the features stay the partition's own (zero-copy) array, so
        # they keep its dtype where the per-row path returns float64 toArray() copies
        if categorical and not nb_classes:
            nb_classes = int(max(int(p.y.max()) for p in parts if len(p))) + 1
        out = []
        for p in parts:
            x = p.x
            if categorical:
                y = np.zeros((len(p), nb_classes))
                y[np.arange(len(p)), p.y.astype(np.int64)] = 1.0
            else:
                y = np.asarray(p.y, dtype=np.float64)
            out.append(ColumnarPartition(x, y))
        return RDD(out, lp_rdd.context)
    if categorical:
        if not nb_classes:
            nb_classes = lp_rdd.map(lambda lp: lp.label).map(int).max() + 1
        return lp_rdd.map(lambda lp: (from_vector(lp.features), encode_label(lp.label, nb_classes)))
    return lp_rdd.map(lambda lp: (from_vector(lp.features), lp.label))
