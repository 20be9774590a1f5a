"""In-process, eager stand-in for Spark's SparkContext / RDD / Broadcast.

There is no JVM: an RDD is a list of partitions (lists) held in host memory,
and partition i is what one logical worker trains on.  The operations keep
Spark's observable semantics that the reference relies on
(SURVEY.md §2.7 'Spark partitioning'):
  * ``parallelize`` cuts the data into ``numSlices`` CONTIGUOUS slices
    (``defaultParallelism`` = N of ``local[N]``);
  * ``repartition(n)`` redistributes round-robin (order is not preserved,
    which is why the reference index-tags predictions: spark_model.py:257-266);
  * ``zipWithIndex`` numbers elements in partition order; ``sortBy`` sorts.
Partitions built from numpy arrays (``to_simple_rdd``, ``parallelize`` of a
``ColumnarPartition``) stay COLUMNAR: a partition is a pair of array views
(features, labels) that behaves like a list of (x, y) tuples for the generic
operations, while the training path hands the arrays straight to the pinned
loader (worker.partition_to_numpy) -- no per-row Python objects, no copies.
"""
from __future__ import annotations

import itertools
import os
import re
from functools import reduce as _reduce
from typing import Any, Callable, Iterable, List, Optional


class SparkConf:
    def __init__(self, loadDefaults=True):
        self._conf = {}

    def setAppName(self, name):
        self._conf["spark.app.name"] = name
        return self

    def setMaster(self, master):
        self._conf["spark.master"] = master
        return self

    def set(self, key, value):
        self._conf[key] = value
        return self

    def get(self, key, default=None):
        return self._conf.get(key, default)

    def getAll(self):
        return list(self._conf.items())


class Broadcast:
    def __init__(self, value):
        self._value = value

    @property
    def value(self):
        return self._value

    def unpersist(self, blocking=False):
        pass

    def destroy(self, blocking=False):
        self._value = None


def _parallelism_from_master(master: str) -> int:
    m = re.match(r"local\[(\d+|\*)\]", master or "")
    if m:
        if m.group(1) == "*":
            return max(1, min(os.cpu_count() or 1, 8))
        return int(m.group(1))
    if master == "local":
        return 1
    return max(1, min(os.cpu_count() or 1, 8))


class SparkContext:
    _active: Optional["SparkContext"] = None

    def __init__(self, master: Optional[str] = None, appName: Optional[str] = None, conf: Optional[SparkConf] = None,
                 **kwargs):
        conf = conf or SparkConf()
        self._conf = conf
        self.master = master or conf.get("spark.master", os.environ.get("ELEPHAS_AMD_MASTER", "local[*]"))
        self.appName = appName or conf.get("spark.app.name", "elephas_amd")
        self.defaultParallelism = _parallelism_from_master(self.master)
        SparkContext._active = self

    @classmethod
    def getOrCreate(cls, conf: Optional[SparkConf] = None) -> "SparkContext":
        if cls._active is None:
            cls._active = SparkContext(conf=conf)
        return cls._active

    def getConf(self):
        return self._conf

    def stop(self):
        if SparkContext._active is self:
            SparkContext._active = None

    def parallelize(self, data: Iterable, numSlices: Optional[int] = None) -> "RDD":
        items = list(data)
        n = numSlices or self.defaultParallelism
        n = max(1, int(n))
        parts = [items[i * len(items) // n:(i + 1) * len(items) // n] for i in range(n)]
        return RDD(parts, self)

    def broadcast(self, value) -> Broadcast:
        return Broadcast(value)

    def emptyRDD(self) -> "RDD":
        return RDD([[]], self)

    def textFile(self, path: str, minPartitions: Optional[int] = None) -> "RDD":
        with open(path, "r") as f:
            lines = [l.rstrip("\n") for l in f]
        return self.parallelize(lines, minPartitions)

    def union(self, rdds):
        parts = []
        for r in rdds:
            parts.extend(r._parts)
        return RDD(parts, self)

    def setLogLevel(self, level):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.stop()


class ColumnarPartition:
    """Rows ``(x[i], y[i])`` of two row-aligned numpy arrays, without per-row objects.

    Sequence protocol (len / iteration / indexing / slicing) so every RDD operation
    that treats a partition as a list of pairs keeps working; ``x`` / ``y`` are the
    zero-copy views the MI355X training path uploads."""

    __slots__ = ("x", "y")

    def __init__(self, x, y):
        if len(x) != len(y):
            raise ValueError("features and labels must have the same number of rows")
        self.x, self.y = x, y

    def __len__(self):
        return len(self.x)

    def __iter__(self):
        return zip(self.x, self.y)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return ColumnarPartition(self.x[i], self.y[i])
        return self.x[i], self.y[i]

    def __bool__(self):
        return len(self.x) > 0

    def __eq__(self, other):
        return list(self) == list(other)

    def __repr__(self):
        return f"ColumnarPartition({len(self)} rows)"


class LabeledPointPartition(ColumnarPartition):
    """Rows ``LabeledPoint(y[i], DenseVector(x[i]))`` of a feature matrix and a label
    vector (the MLlib RDDs of SparkMLlibModel): iterates, indexes and slices as
    LabeledPoint objects built on demand, while the adapters (utils/rdd_utils.py
    lp_to_simple_rdd) convert the arrays in one vectorised step instead of row by row
    (Otto, 61,878 rows: ~100 ms of per-row Python per fit otherwise)."""

    __slots__ = ()

    def __iter__(self):
        from .linalg import DenseVector, LabeledPoint
        return (LabeledPoint(l, DenseVector(r)) for r, l in zip(self.x, self.y))

    def __getitem__(self, i):
        if isinstance(i, slice):
            return LabeledPointPartition(self.x[i], self.y[i])
        from .linalg import DenseVector, LabeledPoint
        return LabeledPoint(self.y[i], DenseVector(self.x[i]))

    def __repr__(self):
        return f"LabeledPointPartition({len(self)} rows)"


def _owned_frozen(a):
    """A read-only copy owned by the partition (the native trainer cache may then keep
    its uploaded shard for as long as the partition lives: worker._DataKey)."""
    import numpy as np
    out = np.array(a, copy=True, order="C")
    out.setflags(write=False)
    return out


def _is_frozen(a) -> bool:
    """No one can write a's bytes through a view: a is an ndarray, it and every array it
    views are read-only, and the chain ends at an array owning its memory (or at an
    immutable ``bytes`` object).  Lists, tensors and arrays over mutable buffers
    (bytearray, mmap, ...) are never frozen.  (An owning array can still be made writeable
    again explicitly; the arrays this module freezes are its own copies.)"""
    import numpy as np
    if not isinstance(a, np.ndarray):
        return False
    while isinstance(a, np.ndarray):
        if a.flags.writeable:
            return False
        a = a.base
    return a is None or isinstance(a, bytes)


def _columnar(parts) -> bool:
    return bool(parts) and all(isinstance(p, ColumnarPartition) for p in parts)


class RDD:
    def __init__(self, partitions: List[list], ctx: Optional[SparkContext] = None):
        self._parts = [p if isinstance(p, ColumnarPartition) else list(p) for p in partitions]
        self.ctx = ctx or SparkContext.getOrCreate()

    @classmethod
    def from_arrays(cls, x, y, num_slices: int, ctx: Optional[SparkContext] = None, snapshot: bool = True,
                    part_cls=None) -> "RDD":
        """``parallelize`` of row-aligned arrays: contiguous columnar slices.  As PySpark's
        ``parallelize`` (which serialises the collection when the RDD is created), the RDD
        holds a read-only snapshot of the arrays -- an edit of the caller's arrays after
        this does not reach it -- so its partitions stay the same frozen arrays for the
        RDD's life and the native trainer keeps their uploaded shards across fits
        (worker._DataKey).  ``snapshot=False``: views of the caller's arrays."""
        if snapshot:
            x, y = _owned_frozen(x), _owned_frozen(y)
        n, k = len(x), max(1, int(num_slices))
        part_cls = part_cls or ColumnarPartition
        return cls([part_cls(x[i * n // k:(i + 1) * n // k], y[i * n // k:(i + 1) * n // k]) for i in range(k)], ctx)

    # ---- structure
    @property
    def context(self):
        return self.ctx

    def getNumPartitions(self) -> int:
        return len(self._parts)

    def glom(self) -> "RDD":
        return RDD([[list(p)] for p in self._parts], self.ctx)

    def partitions(self) -> List[list]:
        """The partitions (columnar ones as zero-copy ColumnarPartition views)."""
        return [p if isinstance(p, ColumnarPartition) else list(p) for p in self._parts]

    def cache(self):
        return self

    persist = cache

    def unpersist(self, blocking=False):
        return self

    # ---- transformations
    def map(self, f, preservesPartitioning=False) -> "RDD":
        return RDD([[f(x) for x in p] for p in self._parts], self.ctx)

    def flatMap(self, f, preservesPartitioning=False) -> "RDD":
        return RDD([[y for x in p for y in f(x)] for p in self._parts], self.ctx)

    def filter(self, f) -> "RDD":
        return RDD([[x for x in p if f(x)] for p in self._parts], self.ctx)

    def mapPartitions(self, f, preservesPartitioning=False) -> "RDD":
        out = []
        for p in self._parts:
            r = f(iter(p))
            out.append(list(r) if r is not None else [])
        return RDD(out, self.ctx)

    def mapPartitionsWithIndex(self, f, preservesPartitioning=False) -> "RDD":
        out = []
        for i, p in enumerate(self._parts):
            r = f(i, iter(p))
            out.append(list(r) if r is not None else [])
        return RDD(out, self.ctx)

    def repartition(self, numPartitions: int) -> "RDD":
        n = max(1, int(numPartitions))
        if _columnar(self._parts):
            # round-robin over the global row order, as below, on the arrays: output
            # partition i takes global rows i, i + n, ...; of input partition j (global
            # offset o_j) that is the strided slice starting at (i - o_j) mod n -- no index
            # arrays, one copy per output partition
            import numpy as np
            frozen = all(_is_frozen(p.x) and _is_frozen(p.y) for p in self._parts)
            memo = getattr(self, "_repart_memo", None)
            if frozen and memo is not None and n in memo:
                return memo[n]   # an RDD is immutable: the same (frozen) output partitions
            kind = type(self._parts[0]) if len({type(p) for p in self._parts}) == 1 else ColumnarPartition
            offs, o = [], 0
            for p in self._parts:
                offs.append(o)
                o += len(p)
            out = []
            for i in range(n):
                xs = [np.asarray(p.x)[(i - oj) % n::n] for p, oj in zip(self._parts, offs)]
                ys = [np.asarray(p.y)[(i - oj) % n::n] for p, oj in zip(self._parts, offs)]
                x = np.concatenate(xs) if len(xs) > 1 else np.array(xs[0])
                y = np.concatenate(ys) if len(ys) > 1 else np.array(ys[0])
                x.setflags(write=False)
                y.setflags(write=False)
                out.append(kind(x, y))
            res = RDD(out, self.ctx)
            if frozen:   # memoised for the last numPartitions only: one extra copy of the data at most
                self._repart_memo = {n: res}
            return res
        parts = [[] for _ in range(n)]
        for i, x in enumerate(itertools.chain.from_iterable(self._parts)):
            parts[i % n].append(x)
        return RDD(parts, self.ctx)

    def coalesce(self, numPartitions: int, shuffle: bool = False) -> "RDD":
        if shuffle:
            return self.repartition(numPartitions)
        n = max(1, min(int(numPartitions), len(self._parts)))
        groups = [self._parts[i * len(self._parts) // n:(i + 1) * len(self._parts) // n] for i in range(n)]
        return RDD([[x for p in g for x in p] for g in groups], self.ctx)

    def zipWithIndex(self) -> "RDD":
        out, k = [], 0
        for p in self._parts:
            q = []
            for x in p:
                q.append((x, k))
                k += 1
            out.append(q)
        return RDD(out, self.ctx)

    def zip(self, other: "RDD") -> "RDD":
        if [len(p) for p in self._parts] != [len(p) for p in other._parts]:
            raise ValueError("Can only zip RDDs with the same number of elements in each partition")
        return RDD([list(zip(a, b)) for a, b in zip(self._parts, other._parts)], self.ctx)

    def sortBy(self, keyfunc, ascending=True, numPartitions=None) -> "RDD":
        items = sorted(self.collect(), key=keyfunc, reverse=not ascending)
        n = numPartitions or len(self._parts)
        return self.ctx.parallelize(items, n)

    def distinct(self, numPartitions=None) -> "RDD":
        seen, out = set(), []
        for x in self.collect():
            k = x if not hasattr(x, "toArray") else x.toArray().tobytes()
            try:
                if k in seen:
                    continue
                seen.add(k)
            except TypeError:
                pass
            out.append(x)
        return self.ctx.parallelize(out, numPartitions or len(self._parts))

    def keys(self):
        return self.map(lambda kv: kv[0])

    def values(self):
        return self.map(lambda kv: kv[1])

    def union(self, other):
        return RDD(self._parts + other._parts, self.ctx)

    def sample(self, withReplacement, fraction, seed=None):
        import random
        rnd = random.Random(seed)
        return RDD([[x for x in p if rnd.random() < fraction] for p in self._parts], self.ctx)

    # ---- actions
    def collect(self) -> list:
        return [x for p in self._parts for x in p]

    def to_arrays(self):
        """(features, labels) of a columnar RDD as two arrays (partition order)."""
        import numpy as np
        if not _columnar(self._parts):
            items = self.collect()
            return np.asarray([a for a, _ in items]), np.asarray([b for _, b in items])
        return np.concatenate([p.x for p in self._parts]), np.concatenate([p.y for p in self._parts])

    def count(self) -> int:
        return sum(len(p) for p in self._parts)

    def first(self):
        for p in self._parts:
            if p:
                return p[0]
        raise ValueError("RDD is empty")

    def take(self, n: int) -> list:
        return list(itertools.islice(itertools.chain.from_iterable(self._parts), n))

    def reduce(self, f):
        items = self.collect()
        if not items:
            raise ValueError("Can not reduce() empty RDD")
        return _reduce(f, items)

    def fold(self, zeroValue, op):
        return _reduce(op, self.collect(), zeroValue)

    def sum(self):
        return sum(self.collect())

    def max(self, key=None):
        return max(self.collect(), key=key) if key else max(self.collect())

    def min(self, key=None):
        return min(self.collect(), key=key) if key else min(self.collect())

    def mean(self):
        items = self.collect()
        return sum(items) / len(items)

    def foreach(self, f):
        for x in self.collect():
            f(x)

    def foreachPartition(self, f):
        for p in self._parts:
            f(iter(p))

    def isEmpty(self) -> bool:
        return self.count() == 0

    def toDF(self, schema=None):
        from .sql import SparkSession
        return SparkSession.builder.getOrCreate().createDataFrame(self, schema)

    def __repr__(self):
        return f"RDD[{self.getNumPartitions()} partitions, {self.count()} elements]"
