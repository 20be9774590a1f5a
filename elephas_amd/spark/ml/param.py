"""``pyspark.ml.param`` (+ the shared column mixins)."""
from ...data.ml import (HasFeaturesCol, HasInputCol, HasLabelCol, HasOutputCol, Param, Params,  # noqa: F401
                        keyword_only)
