"""``pyspark.sql.functions``-shaped column helpers for the host DataFrame.

Covers what the reference tests and examples use on prediction columns
(reference tests/test_ml_model.py:20-27 builds ``argmax`` with
``F.expr('array_position(c, array_max(c)) - 1')``): ``col``, ``lit``, ``udf``,
``array_max``, ``array_position``, ``argmax`` and an ``expr`` that understands the
array_position/array_max idiom plus plain column names.
"""
from __future__ import annotations

import re
from typing import Any, Callable, Union

import numpy as np

from .sql import Column, DoubleType, IntegerType, col  # noqa: F401

_ARGMAX = re.compile(r"^\s*array_position\(\s*(\w+)\s*,\s*array_max\(\s*(\w+)\s*\)\s*\)\s*-\s*1\s*$")
_ARRMAX = re.compile(r"^\s*array_max\(\s*(\w+)\s*\)\s*$")


def _name(c: Union[str, Column]) -> str:
    return c.out_name if isinstance(c, Column) else str(c)


def lit(value: Any) -> Column:
    return Column(repr(value), fn=lambda row: value)


def array_max(c: Union[str, Column]) -> Column:
    n = _name(c)
    return Column(f"array_max({n})", fn=lambda row: float(np.max(np.asarray(row[n]))), dtype=DoubleType())


def argmax(c: Union[str, Column]) -> Column:
    """0-based index of the first maximum of an array column."""
    n = _name(c)
    return Column(f"argmax({n})", fn=lambda row: int(np.argmax(np.asarray(row[n]))), dtype=IntegerType())


def array_position(c: Union[str, Column], value: Any) -> Column:
    """1-based position of ``value`` in an array column (0 when absent), as in Spark SQL."""
    n = _name(c)

    def f(row):
        arr = list(np.asarray(row[n]).ravel())
        v = value.eval(row) if isinstance(value, Column) else value
        return arr.index(v) + 1 if v in arr else 0
    return Column(f"array_position({n})", fn=f, dtype=IntegerType())


def expr(s: str) -> Column:
    m = _ARGMAX.match(s)
    if m and m.group(1) == m.group(2):
        return argmax(m.group(1))
    m = _ARRMAX.match(s)
    if m:
        return array_max(m.group(1))
    if re.match(r"^\s*\w+\s*$", s):
        return col(s.strip())
    raise NotImplementedError(f"expression not supported by the host DataFrame: {s!r}")


def udf(f: Callable = None, returnType=None):
    """Wrap a Python function as a column function: ``udf(fn, DoubleType())(col_a, col_b)``."""
    def wrap(fn):
        def make(*cols):
            names = [_name(c) for c in cols]
            return Column(f"{fn.__name__}({', '.join(names)})", fn=lambda row: fn(*[row[n] for n in names]),
                          dtype=returnType)
        return make
    return wrap(f) if f is not None else wrap
