"""Spark-local semantics of the host data layer (reference tests/utils/test_rdd_utils.py,
tests/ml/test_adapter.py) plus RDD/DataFrame/ML-pipeline behaviour the API relies on."""
import numpy as np
import pytest

from elephas_amd.data import LabeledPoint, SparkContext, SparkSession, Vectors
from elephas_amd.ml import adapter
from elephas_amd.utils import rdd_utils


def test_to_simple_rdd(spark_context):
    rdd = rdd_utils.to_simple_rdd(spark_context, np.ones((5, 10)), np.ones((5,)))
    assert rdd.count() == 5
    first = rdd.first()
    assert first[0].shape == (10,) and first[1] == 1.0


def test_labeled_point_roundtrips(spark_context):
    features = np.ones((2, 10))
    cat = np.asarray([[0, 0, 1.0], [0, 1.0, 0]])
    lp = rdd_utils.to_labeled_point(spark_context, features, cat, True)
    assert lp.count() == 2 and lp.first().label == 2.0 and lp.first().features.shape == (10,)
    x, y = rdd_utils.from_labeled_point(lp, True, 3)
    assert x.shape == features.shape and y.shape == cat.shape
    lp2 = rdd_utils.to_labeled_point(spark_context, features, np.asarray([2.0, 1.0]), False)
    x, y = rdd_utils.from_labeled_point(lp2, False, None)
    assert y.shape == (2,)
    r = rdd_utils.lp_to_simple_rdd(lp, categorical=True)  # nb_classes inferred
    assert r.first()[1].shape == (3,)
    r2 = rdd_utils.lp_to_simple_rdd(lp2, categorical=False, nb_classes=3)
    assert r2.first()[1] == 2.0
    # (n, 1) labels take the columnar path; multi-column labels without ``categorical``
    # take the reference's per-row LabeledPoint construction, which rejects them
    lp3 = rdd_utils.to_labeled_point(spark_context, features, np.asarray([[2.0], [1.0]]), False)
    assert lp3.first().label == 2.0
    with pytest.raises(TypeError):
        rdd_utils.to_labeled_point(spark_context, features, cat, False)


def test_encode_label():
    e = rdd_utils.encode_label(3, 10)
    assert len(e) == 10 and e[3] == 1 and e.sum() == 1


def test_data_frame_adapters(spark_context):
    features = np.ones((2, 10))
    df = adapter.to_data_frame(spark_context, features, np.asarray([[2.0], [1.0]]), categorical=False)
    assert df.count() == 2
    df2 = adapter.to_data_frame(spark_context, features, np.asarray([[0, 0, 1.0], [0, 1.0, 0]]), categorical=True)
    x, y = adapter.from_data_frame(df2, categorical=True, nb_classes=3)
    assert x.shape == (2, 10) and y.shape == (2, 3)
    rdd = adapter.df_to_simple_rdd(adapter.to_data_frame(spark_context, features, np.asarray([2.0, 1.0])), False)
    assert rdd.count() == 2
    renamed = df.withColumnRenamed("features", "f").withColumnRenamed("label", "l")
    r = adapter.df_to_simple_rdd(renamed, False, features_col="f", label_col="l")
    assert r.first()[0].shape == (10,)


def test_parallelize_contiguous_and_repartition(spark_context):
    sc = SparkContext(master="local[4]")
    rdd = sc.parallelize(range(10))
    assert rdd.getNumPartitions() == 4
    assert rdd.glom().collect() == [[0, 1], [2, 3, 4], [5, 6], [7, 8, 9]]
    rp = rdd.repartition(3)
    assert rp.getNumPartitions() == 3 and sorted(rp.collect()) == list(range(10))
    z = rdd.zipWithIndex().collect()
    assert z[3] == (3, 3)
    assert rdd.map(lambda v: v * 2).reduce(lambda a, b: a + b) == 90
    assert rdd.sortBy(lambda v: -v).collect()[0] == 9
    assert sc.parallelize([1, 2]).zip(sc.parallelize([3, 4])).collect() == [(1, 3), (2, 4)]
    assert rdd.mapPartitions(lambda it: [sum(it)]).collect() == [1, 9, 11, 24]


def test_dataframe_sql_and_show(spark_context, capsys):
    spark = SparkSession.builder.getOrCreate()
    df = spark.createDataFrame([(Vectors.dense([1.0, 2.0]), "a"), (Vectors.dense([3.0, 4.0]), "b")],
                               ["features", "category"])
    df.createOrReplaceTempView("t1")
    s = spark.sql("SELECT features AS f, category as c from t1")
    assert s.columns == ["f", "c"] and s.first().c == "a"
    df.show()
    assert "category" in capsys.readouterr().out
    assert df.select("category").distinct().count() == 2


def test_string_indexer_and_scaler_pipeline(spark_context):
    from elephas_amd.data.ml import Pipeline, StandardScaler, StringIndexer, PipelineModel
    spark = SparkSession.builder.getOrCreate()
    rows = [(Vectors.dense([float(i), 2.0 * i]), c) for i, c in enumerate("aabbbc")]
    df = spark.createDataFrame(rows, ["features", "category"])
    si = StringIndexer(inputCol="category", outputCol="idx")
    sc_ = StandardScaler(inputCol="features", outputCol="scaled", withStd=True, withMean=True)
    pm = Pipeline(stages=[si, sc_]).fit(df)
    out = pm.transform(df)
    idx = [r.idx for r in out.collect()]
    assert idx == [1.0, 1.0, 0.0, 0.0, 0.0, 2.0]     # frequency-descending
    sc_vals = np.stack([r.scaled.toArray() for r in out.collect()])
    assert np.allclose(sc_vals.mean(0), 0) and np.allclose(sc_vals.std(0, ddof=1), 1)


def test_metrics():
    from elephas_amd.data.ml import MulticlassMetrics, RegressionMetrics
    sc = SparkContext.getOrCreate()
    m = MulticlassMetrics(sc.parallelize([(0.0, 0.0), (1.0, 1.0), (1.0, 0.0), (2.0, 2.0)]))
    assert m.accuracy == 0.75 and m.precision(1.0) == 0.5 and m.recall(0.0) == 0.5
    assert 0 < m.weightedPrecision <= 1
    r = RegressionMetrics(sc.parallelize([(1.0, 1.0), (2.0, 2.5), (3.0, 2.5)]))
    assert abs(r.meanAbsoluteError - 1 / 3) < 1e-9 and r.r2 < 1


def test_columnar_partitions_match_row_partitions():
    """to_simple_rdd keeps numpy views per partition (no per-row objects) and behaves
    exactly like the list-of-pairs RDD: contiguous slices, round-robin repartition,
    collect order; the training path gets the arrays back without a copy."""
    import numpy as np
    from elephas_amd.data import SparkContext, ColumnarPartition
    from elephas_amd.data.rdd import RDD
    from elephas_amd.utils.rdd_utils import to_simple_rdd
    from elephas_amd.worker import partition_to_numpy
    sc = SparkContext(master="local[3]")
    x = np.arange(22 * 4, dtype=np.float32).reshape(22, 4)
    y = np.arange(22) % 3
    col = to_simple_rdd(sc, x, y)
    rows = RDD([list(p) for p in col.partitions()], sc)          # the row-wise equivalent
    assert all(isinstance(p, ColumnarPartition) for p in col.partitions())
    px, py = partition_to_numpy(col.partitions()[1])
    # a read-only snapshot, as PySpark's parallelize: the training path gets the RDD's own
    # arrays back without a copy, and an edit of the caller's array does not reach them
    assert np.shares_memory(px, col.partitions()[1].x) and px.shape == (7, 4) and not px.flags.writeable
    assert not np.shares_memory(px, x)
    for a, b in ((col, rows), (col.repartition(5), rows.repartition(5))):
        assert a.getNumPartitions() == b.getNumPartitions()
        for pa, pb in zip(a.partitions(), b.partitions()):
            assert len(pa) == len(pb)
            for (xa, ya), (xb, yb) in zip(pa, pb):
                assert np.array_equal(xa, xb) and ya == yb
    assert col.count() == 22 and len(col.collect()) == 22
    xs, ys = col.repartition(4).to_arrays()
    assert sorted(map(tuple, xs.tolist())) == sorted(map(tuple, x.tolist()))
    assert col.map(lambda r: r[1]).collect() == list(y)


def test_trainer_cache_data_key_is_exact():
    """Shards are reused only for the same frozen arrays (an in-place edit of
    a writable array, or a new array at a recycled address, must never hit the cache)."""
    from elephas_amd.worker import _data_key
    from elephas_amd.data.rdd import RDD
    x = np.arange(40, dtype=np.float32).reshape(20, 2)
    y = np.arange(20, dtype=np.float32)
    k1 = _data_key([x], [y], 0.1, [True], True)
    assert k1 != _data_key([x], [y], 0.1, [True], True)      # writable: never reused
    parts = RDD.from_arrays(x, y, 2).repartition(2).partitions()
    xs, ys = [p.x for p in parts], [p.y for p in parts]
    assert not xs[0].flags.writeable
    with pytest.raises(ValueError):
        xs[0][0, 0] = 1.0                                       # frozen partitions
    a = _data_key(xs, ys, 0.1, [True, True], True)
    assert a == _data_key(xs, ys, 0.1, [True, True], True)
    assert a != _data_key(xs, ys, 0.2, [True, True], True)
    copies = [np.array(v) for v in xs]
    for c in copies:
        c.setflags(write=False)
    assert a != _data_key(copies, ys, 0.1, [True, True], True)  # equal bytes, other objects
    x[0, 0] = 99.0                                              # the source edit does not reach
    assert parts[0].x[0, 0] == 0.0                              # the owned partition copy


def test_rdd_snapshot_memoized_conversions_reuse_frozen_arrays():
    """parallelize-style snapshots make an RDD immutable, so its columnar conversions are
    memoised: lp_to_simple_rdd and repartition of the same RDD return the very same
    frozen arrays on every fit (the trainer cache then keeps the uploaded shards), the
    strided repartition equals the row-wise round robin, and an edit of the caller's
    arrays after creating the RDD does not reach it."""
    from elephas_amd.data import SparkContext
    from elephas_amd.data.rdd import RDD
    from elephas_amd.utils.rdd_utils import to_labeled_point, lp_to_simple_rdd
    from elephas_amd.worker import _data_key
    sc = SparkContext(master="local[3]")
    rng = np.random.default_rng(0)
    x = rng.random((23, 5), dtype=np.float32)
    y = rng.integers(0, 4, 23).astype(np.float64)
    lp = to_labeled_point(sc, x, y)
    a = lp_to_simple_rdd(lp, True, 4).repartition(2)
    b = lp_to_simple_rdd(lp, True, 4).repartition(2)
    assert a is b
    xs = [p.x for p in a.partitions()]
    ys = [p.y for p in a.partitions()]
    assert _data_key(xs, ys, 0.1, [True, True], True) == _data_key([p.x for p in b.partitions()],
                                                                    [p.y for p in b.partitions()], 0.1,
                                                                    [True, True], True)
    rows = RDD([list(p) for p in lp_to_simple_rdd(lp, True, 4).partitions()], sc).repartition(2)
    for pa, pb in zip(a.partitions(), rows.partitions()):
        assert len(pa) == len(pb)
        for (xa, ya), (xb, yb) in zip(pa, pb):
            assert np.array_equal(xa, xb) and np.array_equal(ya, yb)
    x[0, 0] = 7.0
    assert lp.partitions()[0].x[0, 0] != 7.0
