"""DataFrame / SparkSession subset (pyspark.sql) backed by the in-process RDD.

Covers what the reference's Spark-ML integration touches
(reference elephas/ml/adapter.py:11-46 createDataFrame / temp view + SQL
``SELECT a AS features, b as label from temp_table``; ml_model.py:191-256
``df.rdd``, ``df.schema``, ``createDataFrame(rdd, schema)``; tests: ``select``,
``withColumnRenamed``, ``show``, ``take``, ``count``, ``distinct``).
"""
from __future__ import annotations

import copy
import re
from typing import Any, Dict, Iterable, List, Optional, Sequence

import numpy as np

from .linalg import DenseVector, LabeledPoint, Vector
from .rdd import RDD, SparkContext


# ------------------------------------------------------------------ types
class DataType:
    def simpleString(self):
        return type(self).__name__.replace("Type", "").lower()

    def __eq__(self, other):
        return type(self) is type(other) and self.__dict__ == other.__dict__

    def __repr__(self):
        return f"{type(self).__name__}()"


class DoubleType(DataType):
    pass


class FloatType(DataType):
    pass


class IntegerType(DataType):
    pass


class LongType(DataType):
    pass


class StringType(DataType):
    pass


class BooleanType(DataType):
    pass


class VectorUDT(DataType):
    def simpleString(self):
        return "vector"


class ArrayType(DataType):
    def __init__(self, elementType, containsNull=True):
        self.elementType = elementType
        self.containsNull = containsNull

    def simpleString(self):
        return f"array<{self.elementType.simpleString()}>"


class StructField:
    def __init__(self, name, dataType, nullable=True, metadata=None):
        self.name, self.dataType, self.nullable = name, dataType, nullable
        self.metadata = metadata or {}

    def __repr__(self):
        return f"StructField({self.name},{self.dataType!r},{self.nullable})"


class StructType(DataType):
    def __init__(self, fields: Optional[List[StructField]] = None):
        self.fields = list(fields or [])

    def add(self, field, data_type=None, nullable=True):
        if isinstance(field, StructField):
            self.fields.append(field)
        else:
            self.fields.append(StructField(field, data_type, nullable))
        return self

    @property
    def names(self):
        return [f.name for f in self.fields]

    def fieldNames(self):
        return self.names

    def __getitem__(self, k):
        if isinstance(k, int):
            return self.fields[k]
        for f in self.fields:
            if f.name == k:
                return f
        raise KeyError(k)

    def __iter__(self):
        return iter(self.fields)

    def __len__(self):
        return len(self.fields)

    def __repr__(self):
        return f"StructType({self.fields!r})"


def _infer_type(v) -> DataType:
    if isinstance(v, Vector):
        return VectorUDT()
    if isinstance(v, (bool, np.bool_)):
        return BooleanType()
    if isinstance(v, (int, np.integer)):
        return LongType()
    if isinstance(v, (float, np.floating)):
        return DoubleType()
    if isinstance(v, str):
        return StringType()
    if isinstance(v, (list, tuple, np.ndarray)):
        return ArrayType(DoubleType())
    return StringType()


# ------------------------------------------------------------------- Row
class Row(tuple):
    """Named tuple with attribute and key access (pyspark.sql.Row)."""

    def __new__(cls, *args, **kwargs):
        if kwargs:
            names = list(kwargs.keys())
            r = tuple.__new__(cls, [kwargs[n] for n in names])
            r.__fields__ = names
            return r
        r = tuple.__new__(cls, args)
        r.__fields__ = None
        return r

    @classmethod
    def from_pairs(cls, names: Sequence[str], values: Sequence[Any]) -> "Row":
        r = tuple.__new__(cls, list(values))
        r.__fields__ = list(names)
        return r

    def __getattr__(self, item):
        if item.startswith("__"):
            raise AttributeError(item)
        f = self.__dict__.get("__fields__")
        if f is not None and item in f:
            return tuple.__getitem__(self, f.index(item))
        raise AttributeError(item)

    def __getitem__(self, k):
        if isinstance(k, str):
            return tuple.__getitem__(self, self.__fields__.index(k))
        return tuple.__getitem__(self, k)

    def asDict(self) -> Dict[str, Any]:
        return dict(zip(self.__fields__, self))

    def __add__(self, other):
        names = list(self.__fields__ or []) + list(getattr(other, "__fields__", None) or
                                                    [f"_{i}" for i in range(len(other))])
        return Row.from_pairs(names, tuple(self) + tuple(other))

    def __repr__(self):
        if self.__fields__:
            return "Row(" + ", ".join(f"{k}={v!r}" for k, v in zip(self.__fields__, self)) + ")"
        return "<Row(" + ", ".join(repr(v) for v in self) + ")>"

    def __reduce__(self):
        return (Row.from_pairs, (self.__fields__, tuple(self)))


# ------------------------------------------------------------- DataFrame
class Column:
    def __init__(self, name: str, alias: Optional[str] = None, fn=None, dtype=None):
        self.name, self._alias, self.fn, self.dtype = name, alias, fn, dtype

    def alias(self, name):
        return Column(self.name, name, self.fn, self.dtype)

    def astype(self, dtype):
        cast = {DoubleType: float, FloatType: float, IntegerType: int, LongType: int, StringType: str}
        f = cast.get(type(dtype), lambda v: v)
        inner = self.fn
        return Column(self.name, self._alias, (lambda row: f(inner(row) if inner else row[self.name])), dtype)

    cast = astype

    @property
    def out_name(self):
        return self._alias or self.name

    def eval(self, row):
        return self.fn(row) if self.fn else row[self.name]


def col(name: str) -> Column:
    return Column(name)


class DataFrame:
    def __init__(self, rows: List[Row], schema: StructType, num_partitions: int = None):
        self._rows = rows
        self.schema = schema
        self._nparts = num_partitions or SparkContext.getOrCreate().defaultParallelism

    @property
    def columns(self) -> List[str]:
        return self.schema.names

    @property
    def rdd(self) -> RDD:
        return SparkContext.getOrCreate().parallelize(self._rows, self._nparts)

    def count(self) -> int:
        return len(self._rows)

    def collect(self) -> List[Row]:
        return list(self._rows)

    def take(self, n: int) -> List[Row]:
        return self._rows[:n]

    def head(self, n: Optional[int] = None):
        return self._rows[0] if n is None else self._rows[:n]

    def first(self) -> Row:
        return self._rows[0]

    def limit(self, n):
        return DataFrame(self._rows[:n], self.schema, self._nparts)

    def _field(self, name):
        return self.schema[name]

    def select(self, *cols) -> "DataFrame":
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = cols[0]
        cs = [c if isinstance(c, Column) else Column(c) for c in cols]
        if len(cs) == 1 and cs[0].name == "*" and cs[0].fn is None:
            return self
        fields = []
        for c in cs:
            if c.fn is None:
                f = copy.copy(self._field(c.name))
                f.name = c.out_name
            else:
                f = StructField(c.out_name, c.dtype or DoubleType())
            fields.append(f)
        names = [f.name for f in fields]
        rows = [Row.from_pairs(names, [c.eval(r) for c in cs]) for r in self._rows]
        return DataFrame(rows, StructType(fields), self._nparts)

    def withColumnRenamed(self, existing: str, new: str) -> "DataFrame":
        fields = []
        for f in self.schema.fields:
            g = copy.copy(f)
            if g.name == existing:
                g.name = new
            fields.append(g)
        names = [f.name for f in fields]
        return DataFrame([Row.from_pairs(names, tuple(r)) for r in self._rows], StructType(fields), self._nparts)

    def withColumn(self, name: str, c: Column) -> "DataFrame":
        vals = [c.eval(r) for r in self._rows]
        names = [n for n in self.columns if n != name] + [name]
        fields = [f for f in self.schema.fields if f.name != name] + \
                 [StructField(name, c.dtype or (_infer_type(vals[0]) if vals else DoubleType()))]
        rows = [Row.from_pairs(names, [r[n] for n in names[:-1]] + [v]) for r, v in zip(self._rows, vals)]
        return DataFrame(rows, StructType(fields), self._nparts)

    def drop(self, *names):
        keep = [n for n in self.columns if n not in names]
        return self.select(*keep)

    def distinct(self) -> "DataFrame":
        seen, out = set(), []
        for r in self._rows:
            key = tuple(v.toArray().tobytes() if isinstance(v, Vector) else
                        (tuple(v) if isinstance(v, list) else v) for v in r)
            if key not in seen:
                seen.add(key)
                out.append(r)
        return DataFrame(out, self.schema, self._nparts)

    def filter(self, fn):
        return DataFrame([r for r in self._rows if fn(r)], self.schema, self._nparts)

    where = filter

    def repartition(self, n):
        return DataFrame(self._rows, self.schema, n)

    def union(self, other):
        return DataFrame(self._rows + other._rows, self.schema, self._nparts)

    def createOrReplaceTempView(self, name: str) -> None:
        SparkSession.builder.getOrCreate()._views[name] = self

    registerTempTable = createOrReplaceTempView

    def printSchema(self):
        print("root")
        for f in self.schema.fields:
            print(f" |-- {f.name}: {f.dataType.simpleString()} (nullable = {str(f.nullable).lower()})")

    def show(self, n: int = 20, truncate=True, vertical=False):
        width = 20 if truncate is True else (int(truncate) if truncate else 10 ** 9)

        def fmt(v):
            if isinstance(v, Vector):
                s = "[" + ",".join(f"{x:g}" for x in v.toArray()) + "]"
            elif isinstance(v, (list, tuple, np.ndarray)):
                s = "[" + ", ".join(f"{x:g}" if isinstance(x, float) else str(x) for x in v) + "]"
            else:
                s = str(v)
            return s if len(s) <= width else s[:max(width - 3, 0)] + "..."
        rows = [[fmt(v) for v in r] for r in self._rows[:n]]
        heads = self.columns
        ws = [max([len(h)] + [len(r[i]) for r in rows]) for i, h in enumerate(heads)]
        line = "+" + "+".join("-" * w for w in ws) + "+"
        print(line)
        print("|" + "|".join(h.rjust(w) for h, w in zip(heads, ws)) + "|")
        print(line)
        for r in rows:
            print("|" + "|".join(v.rjust(w) for v, w in zip(r, ws)) + "|")
        print(line)
        if len(self._rows) > n:
            print(f"only showing top {n} rows")

    def toPandas(self):
        import pandas as pd
        return pd.DataFrame([r.asDict() for r in self._rows], columns=self.columns)

    def __getitem__(self, name):
        return Column(name)

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        if name in self.schema.names:
            return Column(name)
        raise AttributeError(name)

    def __repr__(self):
        return "DataFrame[" + ", ".join(f"{f.name}: {f.dataType.simpleString()}" for f in self.schema.fields) + "]"


# ------------------------------------------------------------ SparkSession
class _Builder:
    def appName(self, name):
        return self

    def master(self, m):
        return self

    def config(self, *a, **k):
        return self

    def enableHiveSupport(self):
        return self

    def getOrCreate(self) -> "SparkSession":
        if SparkSession._active is None:
            SparkSession._active = SparkSession(SparkContext.getOrCreate())
        return SparkSession._active


_SQL_SELECT = re.compile(r"^\s*select\s+(?P<cols>.+?)\s+from\s+(?P<table>\w+)\s*;?\s*$", re.I | re.S)


class SparkSession:
    _active: Optional["SparkSession"] = None
    builder = _Builder()

    def __init__(self, sparkContext: Optional[SparkContext] = None):
        self.sparkContext = sparkContext or SparkContext.getOrCreate()
        self._views: Dict[str, DataFrame] = {}

    def stop(self):
        SparkSession._active = None

    def createDataFrame(self, data, schema=None, samplingRatio=None) -> DataFrame:
        nparts = None
        if isinstance(data, RDD):
            nparts = data.getNumPartitions()
            data = data.collect()
        data = list(data)
        if isinstance(schema, (list, tuple)):
            names = list(schema)
            schema = None
        else:
            names = None
        if data and isinstance(data[0], LabeledPoint):
            names = names or ["label", "features"]
            rows = [Row.from_pairs(names, (lp.label, lp.features)) for lp in data]
            schema = schema or StructType([StructField(names[0], DoubleType()), StructField(names[1], VectorUDT())])
            return DataFrame(rows, schema, nparts)
        if data and isinstance(data[0], Row) and data[0].__fields__ and names is None and schema is None:
            names = list(data[0].__fields__)
        if isinstance(schema, StructType):
            names = schema.names
        if data and isinstance(data[0], dict):
            names = names or list(data[0].keys())
            data = [[d[n] for n in names] for d in data]
        if names is None:
            width = len(data[0]) if data else 0
            names = [f"_{i + 1}" for i in range(width)]
        rows = [Row.from_pairs(names, tuple(r)) for r in data]
        if schema is None:
            first = rows[0] if rows else [None] * len(names)
            schema = StructType([StructField(n, _infer_type(v)) for n, v in zip(names, first)])
        return DataFrame(rows, schema, nparts)

    def sql(self, query: str) -> DataFrame:
        m = _SQL_SELECT.match(query)
        if not m:
            raise NotImplementedError(f"only 'SELECT <cols> FROM <view>' is supported, got: {query}")
        df = self._views[m.group("table")]
        cols = []
        for part in m.group("cols").split(","):
            toks = part.strip().split()
            if len(toks) == 1:
                cols.append(Column(toks[0]))
            elif len(toks) == 3 and toks[1].lower() == "as":
                cols.append(Column(toks[0]).alias(toks[2]))
            else:
                raise NotImplementedError(f"unsupported select item: {part}")
        return df.select(*cols)

    @property
    def read(self):
        return _Reader(self)

    def table(self, name):
        return self._views[name]


class _Reader:
    def __init__(self, spark):
        self.spark = spark

    def csv(self, path, header=False, inferSchema=False):
        import csv
        with open(path) as f:
            rows = list(csv.reader(f))
        names = rows[0] if header else [f"_c{i}" for i in range(len(rows[0]))]
        body = rows[1:] if header else rows
        if inferSchema:
            def conv(v):
                try:
                    return float(v) if any(c in v for c in ".eE") else int(v)
                except ValueError:
                    return v
            body = [[conv(v) for v in r] for r in body]
        return self.spark.createDataFrame(body, names)
