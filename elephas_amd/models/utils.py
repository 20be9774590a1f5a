"""keras.utils subset."""
import numpy as np


def to_categorical(y, num_classes=None, dtype="float32"):
    y = np.asarray(y, dtype="int64").reshape(-1)
    n = int(num_classes) if num_classes is not None else int(y.max()) + 1
    out = np.zeros((y.shape[0], n), dtype=dtype)
    out[np.arange(y.shape[0]), y] = 1
    return out
