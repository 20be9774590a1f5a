"""``pyspark.mllib.evaluation``."""
from ...data.ml import MulticlassMetrics, RegressionMetrics  # noqa: F401
