"""``pyspark.sql.functions``."""
from ...data.functions import argmax, array_max, array_position, col, expr, lit, udf  # noqa: F401
