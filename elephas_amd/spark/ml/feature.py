"""``pyspark.ml.feature``: the preprocessing stages the reference pipelines use."""
from ...data.ml import (StandardScaler, StandardScalerModel, StringIndexer, StringIndexerModel,  # noqa: F401
                        VectorAssembler)
