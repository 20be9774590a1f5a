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
    # a read-only snapshot, as parallelize (RDD.from_arrays)
    return RDD.from_arrays(features, lab, sc.defaultParallelism, sc, part_cls=LabeledPointPartition)


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
    from ..data.rdd import LabeledPointPartition
    parts = lp_rdd.partitions() if hasattr(lp_rdd, "partitions") else None
    if parts and all(isinstance(p, LabeledPointPartition) for p in parts):
        from ..data.rdd import _is_frozen
        frozen = all(_is_frozen(p.x) and _is_frozen(p.y) for p in parts)
        memo = getattr(lp_rdd, "_lp_simple_memo", None) if frozen else None
        key = (bool(categorical), nb_classes)
        if memo is not None and key in memo:
            return memo[key]   # the same frozen arrays as the previous conversion of this RDD
        res = _lp_columnar(lp_rdd, parts, categorical, nb_classes)
        if frozen:
            if memo is None:
                memo = lp_rdd._lp_simple_memo = {}
            memo[key] = res
        return res
    if categorical:
        if not nb_classes:
            nb_classes = lp_rdd.map(lambda lp: lp.label).map(int).max() + 1
        return lp_rdd.map(lambda lp: (from_vector(lp.features), encode_label(lp.label, nb_classes)))
    return lp_rdd.map(lambda lp: (from_vector(lp.features), lp.label))


def _lp_columnar(lp_rdd, parts, categorical, nb_classes):
    """Columnar LabeledPoints -> (features, label) partitions as arrays: the same pairs as
    the per-row path; the features stay the partition's own array (no copy, its dtype,
    where the per-row path returns float64 toArray() copies)."""
    from ..data.rdd import ColumnarPartition, RDD
    if categorical and not nb_classes:
        nb_classes = int(max(int(p.y.max()) for p in parts if len(p))) + 1
    out = []
    for p in parts:
        if categorical:
            y = np.zeros((len(p), nb_classes))
            y[np.arange(len(p)), p.y.astype(np.int64)] = 1.0
            y.setflags(write=False)
        else:
            y = np.asarray(p.y, dtype=np.float64)
        out.append(ColumnarPartition(p.x, y))
    return RDD(out, lp_rdd.context)
