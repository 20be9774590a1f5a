"""``pyspark.ml``: Pipeline / PipelineModel / Estimator / Transformer / Model."""
from ...data.ml import Estimator, Model, Pipeline, PipelineModel, Transformer  # noqa: F401
from . import feature, linalg, param  # noqa: F401
