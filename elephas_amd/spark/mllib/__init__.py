"""``pyspark.mllib``."""
from . import evaluation, linalg, regression  # noqa: F401
