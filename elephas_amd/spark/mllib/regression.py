"""``pyspark.mllib.regression``."""
from ...data.linalg import LabeledPoint  # noqa: F401
