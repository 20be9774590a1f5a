"""Element-wise arithmetic over lists of parameter arrays
(reference elephas/utils/functional_utils.py:6-43).  The device-side
equivalents on the packed flat vector are the ``_C.sub``/``axpby``/``ps_sub``
kernels (csrc/kernels/flat.hip)."""
from typing import List

import numpy as np


def add_params(param_list_left: List[np.ndarray], param_list_right: List[np.ndarray]) -> List[np.ndarray]:
    return [x + y for x, y in zip(param_list_left, param_list_right)]


def subtract_params(param_list_left: List[np.ndarray], param_list_right: List[np.ndarray]) -> List[np.ndarray]:
    return [x - y for x, y in zip(param_list_left, param_list_right)]


def get_neutral(array_list: List[np.ndarray]) -> List[np.ndarray]:
    return [np.zeros_like(x) for x in array_list]


def divide_by(array_list: List[np.ndarray], num_workers: int) -> List[np.ndarray]:
    return [x / num_workers for x in array_list]
