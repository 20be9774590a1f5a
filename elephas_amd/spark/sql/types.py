"""``pyspark.sql.types``."""
from ...data.sql import (ArrayType, BooleanType, DataType, DoubleType, FloatType, IntegerType,  # noqa: F401
                         LongType, StringType, StructField, StructType)
