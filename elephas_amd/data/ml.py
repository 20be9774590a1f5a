"""pyspark.ml surface used by the reference's Spark-ML integration
(reference elephas/ml_model.py:25-29 Estimator/Model/Has*Col/DefaultParams*,
elephas/ml/params.py Param mixins, examples/ml_pipeline_otto.py StringIndexer +
StandardScaler + Pipeline, tests/test_ml_model.py MulticlassMetrics /
RegressionMetrics / ``pipeline.save``).
"""
from __future__ import annotations

import copy
import functools
import json
import math
import os
import uuid
from typing import Any, Dict, List, Optional

import numpy as np

from .linalg import DenseVector, Vector
from .sql import DataFrame, DoubleType, Row, StructField, StructType, VectorUDT


# ------------------------------------------------------------------ params
class Param:
    def __init__(self, parent, name: str, doc: str = "", typeConverter=None):
        self.parent = getattr(parent, "uid", "undefined")
        self.name = name
        self.doc = doc
        self.typeConverter = typeConverter or (lambda v: v)

    def __hash__(self):
        return hash((self.parent, self.name))

    def __eq__(self, other):
        return isinstance(other, Param) and self.parent == other.parent and self.name == other.name

    def __repr__(self):
        return f"Param(parent={self.parent!r}, name={self.name!r})"


def keyword_only(func):
    @functools.wraps(func)
    def wrapper(self, *args, **kwargs):
        if args:
            raise TypeError(f"Method {func.__name__} forces keyword arguments.")
        self._input_kwargs = kwargs
        return func(self, **kwargs)
    return wrapper


class Params:
    def __init__(self):
        if not hasattr(self, "uid"):
            self.uid = f"{type(self).__name__}_{uuid.uuid4().hex[:12]}"
        if not hasattr(self, "_paramMap"):
            self._paramMap: Dict[Param, Any] = {}
            self._defaultParamMap: Dict[Param, Any] = {}

    @property
    def params(self) -> List[Param]:
        return [getattr(self, a) for a in dir(type(self)) if False] + \
               [v for v in self.__dict__.values() if isinstance(v, Param)]

    def _resolve(self, p):
        if isinstance(p, Param):
            return p
        if isinstance(p, str):
            v = self.__dict__.get(p)
            if isinstance(v, Param):
                return v
        raise AttributeError(f"{type(self).__name__} has no param {p!r}")

    def hasParam(self, name: str) -> bool:
        return isinstance(self.__dict__.get(name), Param)

    def getParam(self, name):
        return self._resolve(name)

    def isSet(self, p) -> bool:
        return self._resolve(p) in self._paramMap

    def hasDefault(self, p) -> bool:
        return self._resolve(p) in self._defaultParamMap

    def isDefined(self, p) -> bool:
        return self.isSet(p) or self.hasDefault(p)

    def getOrDefault(self, p):
        p = self._resolve(p)
        if p in self._paramMap:
            return self._paramMap[p]
        if p in self._defaultParamMap:
            return self._defaultParamMap[p]
        raise KeyError(f"Param {p.name} has neither a set value nor a default")

    def _set(self, **kwargs):
        for k, v in kwargs.items():
            p = self._resolve(k)
            self._paramMap[p] = p.typeConverter(v) if v is not None else v
        return self

    def set(self, param, value):
        self._paramMap[self._resolve(param)] = value
        return self

    def _setDefault(self, **kwargs):
        for k, v in kwargs.items():
            self._defaultParamMap[self._resolve(k)] = v
        return self

    def clear(self, param):
        self._paramMap.pop(self._resolve(param), None)

    def extractParamMap(self, extra=None) -> Dict[Param, Any]:
        d = dict(self._defaultParamMap)
        d.update(self._paramMap)
        if extra:
            d.update(extra)
        return d

    def explainParams(self) -> str:
        return "\n".join(f"{p.name}: {p.doc}" for p in self.params)

    def copy(self, extra=None):
        c = copy.copy(self)
        c._paramMap = dict(self._paramMap)
        if extra:
            c._paramMap.update(extra)
        return c


class HasFeaturesCol(Params):
    def __init__(self):
        super().__init__()
        self.featuresCol = Param(self, "featuresCol", "features column name")
        self._setDefault(featuresCol="features")

    def setFeaturesCol(self, value):
        return self._set(featuresCol=value)

    def getFeaturesCol(self):
        return self.getOrDefault(self.featuresCol)


class HasLabelCol(Params):
    def __init__(self):
        super().__init__()
        self.labelCol = Param(self, "labelCol", "label column name")
        self._setDefault(labelCol="label")

    def setLabelCol(self, value):
        return self._set(labelCol=value)

    def getLabelCol(self):
        return self.getOrDefault(self.labelCol)


class HasOutputCol(Params):
    def __init__(self):
        super().__init__()
        self.outputCol = Param(self, "outputCol", "output column name")
        self._setDefault(outputCol=f"{self.uid}__output")

    def setOutputCol(self, value):
        return self._set(outputCol=value)

    def getOutputCol(self):
        return self.getOrDefault(self.outputCol)


class HasInputCol(Params):
    def __init__(self):
        super().__init__()
        self.inputCol = Param(self, "inputCol", "input column name")

    def setInputCol(self, value):
        return self._set(inputCol=value)

    def getInputCol(self):
        return self.getOrDefault(self.inputCol)


# --------------------------------------------------------- persistence mix
def _jsonable(v):
    try:
        json.dumps(v)
        return True
    except (TypeError, ValueError):
        return False


class DefaultParamsWritable:
    def write(self):
        return _Writer(self)

    def save(self, path: str):
        self.write().save(path)


class _Writer:
    def __init__(self, inst):
        self.inst = inst
        self._overwrite = False

    def overwrite(self):
        self._overwrite = True
        return self

    def save(self, path):
        if os.path.exists(path) and not self._overwrite and os.listdir(path):
            raise FileExistsError(f"Path {path} already exists. Use write().overwrite().save(path)")
        _save_instance(self.inst, path)


def _save_instance(inst, path):
    os.makedirs(os.path.join(path, "metadata"), exist_ok=True)
    params = {p.name: v for p, v in inst._paramMap.items() if _jsonable(v)}
    defaults = {p.name: v for p, v in inst._defaultParamMap.items() if _jsonable(v)}
    meta = {"class": f"{type(inst).__module__}.{type(inst).__name__}", "uid": inst.uid,
            "paramMap": params, "defaultParamMap": defaults}
    if hasattr(inst, "_extra_state"):
        meta["state"] = inst._extra_state()
    stages = getattr(inst, "stages", None)
    if stages is not None and isinstance(stages, list):
        meta["stageUids"] = []
        for i, s in enumerate(stages):
            sp = os.path.join(path, "stages", f"{i}_{s.uid}")
            _save_instance(s, sp)
            meta["stageUids"].append(f"{i}_{s.uid}")
    with open(os.path.join(path, "metadata", "part-00000"), "w") as f:
        json.dump(meta, f)


def _load_instance(path):
    import importlib
    with open(os.path.join(path, "metadata", "part-00000")) as f:
        meta = json.load(f)
    mod, _, cls = meta["class"].rpartition(".")
    klass = getattr(importlib.import_module(mod), cls)
    if "stageUids" in meta:
        stages = [_load_instance(os.path.join(path, "stages", s)) for s in meta["stageUids"]]
        inst = klass(stages=stages)
    else:
        inst = klass()
    inst.uid = meta["uid"]
    for k, v in meta.get("paramMap", {}).items():
        if inst.hasParam(k):
            inst._paramMap[inst.getParam(k)] = v
    if "state" in meta and hasattr(inst, "_load_state"):
        inst._load_state(meta["state"])
    return inst


class DefaultParamsReadable:
    @classmethod
    def load(cls, path):
        return _load_instance(path)

    @classmethod
    def read(cls):
        return _Reader()


class _Reader:
    def load(self, path):
        return _load_instance(path)


# ---------------------------------------------------------------- stages
class Transformer(Params):
    def transform(self, dataset: DataFrame, params=None) -> DataFrame:
        inst = self.copy(params) if params else self
        return inst._transform(dataset)

    def _transform(self, dataset):
        raise NotImplementedError


class Estimator(Params):
    def fit(self, dataset: DataFrame, params=None):
        inst = self.copy(params) if params else self
        return inst._fit(dataset)

    def _fit(self, dataset):
        raise NotImplementedError


class Model(Transformer):
    pass


class Pipeline(Estimator, DefaultParamsReadable, DefaultParamsWritable):
    def __init__(self, stages=None):
        super().__init__()
        self.stages = list(stages or [])

    def getStages(self):
        return self.stages

    def setStages(self, stages):
        self.stages = list(stages)
        return self

    def _fit(self, df):
        fitted = []
        last_est = max([i for i, s in enumerate(self.stages) if isinstance(s, Estimator)], default=-1)
        for i, s in enumerate(self.stages):
            if isinstance(s, Estimator):
                m = s.fit(df)
                fitted.append(m)
                if i < last_est:
                    df = m.transform(df)
            else:
                fitted.append(s)
                if i < last_est:
                    df = s.transform(df)
        return PipelineModel(fitted)


class PipelineModel(Model, DefaultParamsReadable, DefaultParamsWritable):
    def __init__(self, stages=None):
        super().__init__()
        self.stages = list(stages or [])

    def _transform(self, df):
        for s in self.stages:
            df = s.transform(df)
        return df


# ------------------------------------------------------------- features
def _vec(v) -> np.ndarray:
    return v.toArray() if isinstance(v, Vector) else np.asarray(v, dtype=np.float64)


class StringIndexer(Estimator, HasInputCol, HasOutputCol, DefaultParamsReadable, DefaultParamsWritable):
    """Labels -> indices ordered by descending frequency (ties: alphabetical)."""

    @keyword_only
    def __init__(self, inputCol=None, outputCol=None, handleInvalid="error", stringOrderType="frequencyDesc"):
        super().__init__()
        self.handleInvalid = Param(self, "handleInvalid", "")
        self.stringOrderType = Param(self, "stringOrderType", "")
        self._setDefault(handleInvalid="error", stringOrderType="frequencyDesc")
        self._set(**{k: v for k, v in self._input_kwargs.items() if v is not None})

    def _fit(self, df):
        col = self.getInputCol()
        counts: Dict[Any, int] = {}
        for r in df.collect():
            counts[r[col]] = counts.get(r[col], 0) + 1
        order = self.getOrDefault(self.stringOrderType)
        keys = list(counts)
        if order == "frequencyDesc":
            keys.sort(key=lambda k: (-counts[k], str(k)))
        elif order == "frequencyAsc":
            keys.sort(key=lambda k: (counts[k], str(k)))
        elif order == "alphabetDesc":
            keys.sort(key=str, reverse=True)
        else:
            keys.sort(key=str)
        m = StringIndexerModel(labels=[str(k) for k in keys])
        m._set(inputCol=col, outputCol=self.getOutputCol())
        return m


class StringIndexerModel(Model, HasInputCol, HasOutputCol, DefaultParamsReadable, DefaultParamsWritable):
    def __init__(self, labels=None):
        super().__init__()
        self.labels = list(labels or [])

    def _extra_state(self):
        return {"labels": self.labels}

    def _load_state(self, st):
        self.labels = st["labels"]

    def _transform(self, df):
        idx = {l: float(i) for i, l in enumerate(self.labels)}
        col, out = self.getInputCol(), self.getOutputCol()
        names = df.columns + [out]
        rows = [Row.from_pairs(names, tuple(r) + (idx[str(r[col])],)) for r in df.collect()]
        return DataFrame(rows, StructType(list(df.schema.fields) + [StructField(out, DoubleType())]), df._nparts)


class StandardScaler(Estimator, HasInputCol, HasOutputCol, DefaultParamsReadable, DefaultParamsWritable):
    """Spark semantics: unbiased (n-1) standard deviation; withMean default False."""

    @keyword_only
    def __init__(self, withMean=False, withStd=True, inputCol=None, outputCol=None):
        super().__init__()
        self.withMean = Param(self, "withMean", "")
        self.withStd = Param(self, "withStd", "")
        self._setDefault(withMean=False, withStd=True)
        self._set(**{k: v for k, v in self._input_kwargs.items() if v is not None})

    def _fit(self, df):
        X = np.stack([_vec(r[self.getInputCol()]) for r in df.collect()])
        mean = X.mean(0)
        std = X.std(0, ddof=1) if len(X) > 1 else np.zeros(X.shape[1])
        m = StandardScalerModel(mean=mean.tolist(), std=std.tolist())
        m._set(inputCol=self.getInputCol(), outputCol=self.getOutputCol(),
               withMean=self.getOrDefault(self.withMean), withStd=self.getOrDefault(self.withStd))
        return m


class StandardScalerModel(Model, HasInputCol, HasOutputCol, DefaultParamsReadable, DefaultParamsWritable):
    def __init__(self, mean=None, std=None):
        super().__init__()
        self.withMean = Param(self, "withMean", "")
        self.withStd = Param(self, "withStd", "")
        self._setDefault(withMean=False, withStd=True)
        self.mean = DenseVector(mean or [])
        self.std = DenseVector(std or [])

    def _extra_state(self):
        return {"mean": self.mean.toArray().tolist(), "std": self.std.toArray().tolist()}

    def _load_state(self, st):
        self.mean, self.std = DenseVector(st["mean"]), DenseVector(st["std"])

    def _transform(self, df):
        mu, sd = self.mean.toArray(), self.std.toArray()
        inv = np.where(sd > 0, 1.0 / np.where(sd > 0, sd, 1.0), 0.0)
        wm, ws = self.getOrDefault(self.withMean), self.getOrDefault(self.withStd)
        col, out = self.getInputCol(), self.getOutputCol()
        names = df.columns + [out]
        rows = []
        for r in df.collect():
            v = _vec(r[col]).copy()
            if wm:
                v = v - mu
            if ws:
                v = v * inv
            rows.append(Row.from_pairs(names, tuple(r) + (DenseVector(v),)))
        return DataFrame(rows, StructType(list(df.schema.fields) + [StructField(out, VectorUDT())]), df._nparts)


class VectorAssembler(Transformer, HasOutputCol, DefaultParamsReadable, DefaultParamsWritable):
    @keyword_only
    def __init__(self, inputCols=None, outputCol=None, handleInvalid="error"):
        super().__init__()
        self.inputCols = Param(self, "inputCols", "")
        self._set(**{k: v for k, v in self._input_kwargs.items() if v is not None and k != "handleInvalid"})

    def _transform(self, df):
        cols = self.getOrDefault(self.inputCols)
        out = self.getOutputCol()
        names = df.columns + [out]
        rows = []
        for r in df.collect():
            parts = [np.atleast_1d(_vec(r[c])) for c in cols]
            rows.append(Row.from_pairs(names, tuple(r) + (DenseVector(np.concatenate(parts)),)))
        return DataFrame(rows, StructType(list(df.schema.fields) + [StructField(out, VectorUDT())]), df._nparts)


# ------------------------------------------------------------ evaluation
class MulticlassMetrics:
    """pyspark.mllib.evaluation.MulticlassMetrics over an RDD of (prediction, label)."""

    def __init__(self, predictionAndLabels):
        pl = predictionAndLabels.collect() if hasattr(predictionAndLabels, "collect") else list(predictionAndLabels)
        self._p = np.array([float(a) for a, _ in pl])
        self._l = np.array([float(b) for _, b in pl])
        self.labels = np.unique(np.concatenate([self._l, self._p])) if len(pl) else np.array([])

    @property
    def accuracy(self) -> float:
        return float((self._p == self._l).mean()) if len(self._l) else 0.0

    def confusionMatrix(self):
        from .linalg import DenseMatrix
        labs = list(self.labels)
        m = np.zeros((len(labs), len(labs)))
        for p, l in zip(self._p, self._l):
            m[labs.index(l), labs.index(p)] += 1
        return DenseMatrix(len(labs), len(labs), m.T.reshape(-1))

    def truePositiveRate(self, label):
        return self.recall(label)

    def falsePositiveRate(self, label):
        neg = self._l != label
        return float(((self._p == label) & neg).sum() / max(neg.sum(), 1))

    def precision(self, label=None) -> float:
        if label is None:  # Spark 1.x/2.x overall precision == accuracy
            return self.accuracy
        pred = self._p == label
        return float((pred & (self._l == label)).sum() / pred.sum()) if pred.sum() else 0.0

    def recall(self, label=None) -> float:
        if label is None:
            return self.accuracy
        act = self._l == label
        return float((act & (self._p == label)).sum() / act.sum()) if act.sum() else 0.0

    def fMeasure(self, label=None, beta=1.0) -> float:
        if label is None:
            return self.accuracy
        p, r = self.precision(label), self.recall(label)
        b2 = beta * beta
        return (1 + b2) * p * r / (b2 * p + r) if (p + r) > 0 else 0.0

    def _weighted(self, fn):
        tot = len(self._l)
        return float(sum(fn(l) * (self._l == l).sum() / tot for l in np.unique(self._l))) if tot else 0.0

    @property
    def weightedPrecision(self):
        return self._weighted(self.precision)

    @property
    def weightedRecall(self):
        return self._weighted(self.recall)

    def weightedFMeasure(self, beta=1.0):
        return self._weighted(lambda l: self.fMeasure(l, beta))

    @property
    def weightedTruePositiveRate(self):
        return self.weightedRecall

    @property
    def weightedFalsePositiveRate(self):
        return self._weighted(self.falsePositiveRate)


class RegressionMetrics:
    """pyspark.mllib.evaluation.RegressionMetrics over an RDD of (prediction, observation)."""

    def __init__(self, predictionAndObservations):
        po = predictionAndObservations.collect() if hasattr(predictionAndObservations, "collect") \
            else list(predictionAndObservations)
        self._p = np.array([float(a) for a, _ in po])
        self._o = np.array([float(b) for _, b in po])

    @property
    def meanSquaredError(self):
        return float(np.mean((self._p - self._o) ** 2))

    @property
    def rootMeanSquaredError(self):
        return math.sqrt(self.meanSquaredError)

    @property
    def meanAbsoluteError(self):
        return float(np.mean(np.abs(self._p - self._o)))

    @property
    def r2(self):
        ss_res = np.sum((self._o - self._p) ** 2)
        ss_tot = np.sum((self._o - self._o.mean()) ** 2)
        return float(1 - ss_res / ss_tot) if ss_tot > 0 else 0.0

    @property
    def explainedVariance(self):
        return float(np.mean((self._p - self._o.mean()) ** 2))
