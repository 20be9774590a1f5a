"""``pyspark.sql``."""
from ...data.sql import Column, DataFrame, Row, SparkSession  # noqa: F401
from . import functions, types  # noqa: F401
