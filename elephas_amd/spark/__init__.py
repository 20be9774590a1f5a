"""``pyspark``-shaped namespace over the host data layer (no JVM).

Reference scripts and notebooks import ``pyspark``, ``pyspark.sql``,
``pyspark.ml`` and ``pyspark.mllib`` (reference examples/*.py); with this
package they port by replacing the ``pyspark`` prefix with ``elephas_amd.spark``.
Everything here re-exports ``elephas_amd.data``.
"""
from ..data.rdd import RDD, Broadcast, SparkConf, SparkContext  # noqa: F401
