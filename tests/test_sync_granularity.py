"""Synchronous-mode extensions: averaging granularity
('fit' = reference, 'epoch', 'batch' = per-step gradient all-reduce), resumable
checkpoints, and the fit metrics / tracing hooks."""
import json
import os

import numpy as np
import pytest

from elephas_amd.models import Dense, Sequential
from elephas_amd.models.optimizers import SGD, Adam
from elephas_amd.spark_model import SparkModel, load_spark_model
from elephas_amd.worker import SparkWorker


def _model(opt=None):
    from elephas_amd.models import initializers
    from elephas_amd.models.layers import clear_session
    clear_session()
    initializers.set_seed(5)
    m = Sequential([Dense(8, input_dim=5, activation="tanh"), Dense(3, activation="softmax")])
    m.compile(opt or SGD(0.1), "categorical_crossentropy", ["acc"])
    return m


def _data(n=120, seed=1):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(n, 5)).astype(np.float32)
    y = np.eye(3, dtype=np.float32)[rng.integers(0, 3, n)]
    return x, y


def _train_alone(w0, part, epochs, bs=10):
    m = _model()
    m.set_weights(w0)
    w = SparkWorker(m.to_json(), w0, {"epochs": epochs, "batch_size": bs, "shuffle": False}, SGD(0.1),
                    "categorical_crossentropy", [], {})
    d = next(w.train(iter(part)))[0]
    return [a - b for a, b in zip(w0, d)]


def test_epoch_granularity_averages_every_epoch(spark_context):
    x, y = _data()
    m = _model()
    w0 = m.get_weights()
    rdd = spark_context.parallelize(list(zip(x, y)), 3)
    parts = rdd.partitions()
    sm = SparkModel(m, mode="synchronous", sync_granularity="epoch")
    sm.fit(rdd, epochs=2, batch_size=10, verbose=0, shuffle=False)
    # reference: average after epoch 1, then every worker continues from the mean.
    # SGD without momentum has no optimizer state, so per-epoch restarts are exact.
    w = w0
    for _ in range(2):
        ws = [_train_alone(w, p, 1) for p in parts]
        w = [sum(a[i] for a in ws) / len(ws) for i in range(len(w0))]
    for a, b in zip(sm.master_network.get_weights(), w):
        assert np.allclose(a, b, atol=1e-6)
    assert sm.get_config()["sync_granularity"] == "epoch"
    assert len(sm.training_histories) == 3 and len(sm.training_histories[0]["loss"]) == 2


def test_batch_granularity_identical_shards_equals_single_worker(spark_context):
    """Averaging identical gradients changes nothing: N workers on copies of the
    same shard == one worker on that shard."""
    x, y = _data(60)
    m = _model(Adam(0.01))
    w0 = m.get_weights()
    rdd = spark_context.parallelize(list(zip(x, y)) * 2, 2)   # partition 0 == partition 1
    sm = SparkModel(m, mode="synchronous", sync_granularity="batch")
    sm.fit(rdd, epochs=3, batch_size=16, verbose=0, shuffle=False)
    single = _model(Adam(0.01))
    single.set_weights(w0)
    single.fit(x, y, epochs=3, batch_size=16, verbose=0, shuffle=False)
    for a, b in zip(sm.master_network.get_weights(), single.get_weights()):
        assert np.allclose(a, b, atol=1e-5)


def test_checkpoint_resume_matches_uninterrupted_run(tmp_path, spark_context):
    x, y = _data()
    rdd = spark_context.parallelize(list(zip(x, y)), 3)
    full = SparkModel(_model(Adam(0.01)), mode="synchronous", sync_granularity="epoch")
    full.fit(rdd, epochs=3, batch_size=10, verbose=0, shuffle=False)

    ck = str(tmp_path / "ck")
    part1 = SparkModel(_model(Adam(0.01)), mode="synchronous", sync_granularity="epoch")
    part1.fit(rdd, epochs=2, batch_size=10, verbose=0, shuffle=False, checkpoint_dir=ck)
    meta = json.load(open(os.path.join(ck, "checkpoint.json")))
    assert meta == {"epoch": 2, "epochs": 2}
    # the checkpointed model is a regular Elephas HDF5 file
    loaded = load_spark_model(os.path.join(ck, "model.h5"))
    for a, b in zip(loaded.master_network.get_weights(), part1.master_network.get_weights()):
        assert np.allclose(a, b)
    # a fresh job resumes at epoch 2 (weights AND Adam moments / iteration counters)
    part2 = SparkModel(_model(Adam(0.01)), mode="synchronous", sync_granularity="epoch")
    part2.fit(rdd, epochs=3, batch_size=10, verbose=0, shuffle=False, checkpoint_dir=ck, resume=True)
    for a, b in zip(part2.master_network.get_weights(), full.master_network.get_weights()):
        assert np.allclose(a, b, atol=1e-6)
    assert json.load(open(os.path.join(ck, "checkpoint.json")))["epoch"] == 3


def test_fit_metrics_and_jsonl(tmp_path, spark_context):
    x, y = _data()
    path = str(tmp_path / "m.jsonl")
    sm = SparkModel(_model(), mode="synchronous", metrics_path=path)
    sm.fit(spark_context.parallelize(list(zip(x, y)), 2), epochs=2, batch_size=10, verbose=0)
    m = sm.metrics
    assert m["workers"] == 2 and m["epochs"] == 2 and m["samples"] == 240 and m["samples_per_sec"] > 0
    assert {"broadcast", "setup", "train", "allreduce", "gather_histories"} <= set(m["phases"])
    rec = [json.loads(l) for l in open(path)]
    assert rec[-1]["event"] == "fit" and rec[-1]["samples"] == 240


def test_invalid_granularity():
    with pytest.raises(ValueError):
        SparkModel(_model(), mode="synchronous", sync_granularity="step")


def test_profiling_primitives(tmp_path):
    from elephas_amd.profiling import MetricsLogger, PhaseTimer, mark, trace_range
    calls = []
    t = PhaseTimer(sync=lambda: calls.append(1))
    with t.phase("a"):
        with trace_range("inner"):
            mark("m")
    with t.phase("a"):
        pass
    assert t.counts["a"] == 2 and t.totals["a"] >= 0 and len(calls) == 4
    lg = MetricsLogger(str(tmp_path / "x" / "log.jsonl"), rank=0)
    lg.log("step", ms=1.5)
    MetricsLogger(str(tmp_path / "y.jsonl"), rank=1).log("step")   # only rank 0 writes
    assert json.loads(open(tmp_path / "x" / "log.jsonl").read())["ms"] == 1.5
    assert not (tmp_path / "y.jsonl").exists()
