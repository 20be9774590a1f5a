"""Multi-process data parallelism on CPU: 2 ranks over gloo (the GPU job uses the
same code over RCCL).  Checks that (a) synchronous averaging across ranks equals
the single-process average over the same partitions, (b) every rank ends with
identical master weights, (c) distributed predict/evaluate match local ones, and
(d) the async parameter server works across processes (rank 0 hosts it)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data():
    rng = np.random.default_rng(3)
    x = rng.normal(size=(400, 12)).astype(np.float32)
    y = np.eye(3, dtype=np.float32)[rng.integers(0, 3, 400)]
    return x, y


def _model():
    from elephas_amd.models import Sequential, Dense
    from elephas_amd.models.optimizers import SGD
    from elephas_amd.models.layers import clear_session
    from elephas_amd.models import initializers
    clear_session()
    initializers.set_seed(11)
    m = Sequential([Dense(16, input_dim=12, activation="relu"), Dense(3, activation="softmax")])
    m.compile(SGD(0.05), "categorical_crossentropy", ["acc"])
    return m


def _worker(rank, world, port, mode, ps_mode, out_dir, gran="fit"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SPARK_LOCAL_IP="127.0.0.1", CUDA_VISIBLE_DEVICES="",
                      HIP_VISIBLE_DEVICES="")
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from elephas_amd import config
    config.set_device("cpu")
    from elephas_amd.data import SparkContext
    from elephas_amd.spark_model import SparkModel
    from elephas_amd.utils.rdd_utils import to_simple_rdd
    x, y = _data()
    sc = SparkContext(master="local[4]")
    m = _model()
    sm = SparkModel(m, mode=mode, parameter_server_mode=ps_mode, port=port + 1, sync_granularity=gran)
    sm.fit(to_simple_rdd(sc, x, y), epochs=2, batch_size=16, verbose=0, shuffle=False)
    preds = np.stack(sm.predict(x[:50]))
    ev = sm.evaluate(x, y)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), *sm.master_network.get_weights(), preds=preds,
             ev=np.asarray(ev), nh=len(sm.training_histories))
    dist.barrier()
    dist.destroy_process_group()


def _run(mode, ps_mode, tmp_path, world=2, gran="fit"):
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, mode, ps_mode, str(tmp_path), gran), nprocs=world, join=True,
                       start_method="spawn")
    return [np.load(tmp_path / f"r{r}.npz") for r in range(world)]


@pytest.mark.parametrize("gran", ["fit", "batch"])
def test_sync_two_ranks_equals_single_process(tmp_path, gran):
    outs = _run("synchronous", "http", tmp_path, gran=gran)
    a, b = outs
    for k in a.files:
        assert np.array_equal(a[k], b[k]), k
    assert int(a["nh"]) == 4          # histories of all 4 partitions gathered on every rank
    # single-process reference over the same 4 partitions
    from elephas_amd import config
    config.set_device("cpu")
    from elephas_amd.data import SparkContext
    from elephas_amd.spark_model import SparkModel
    from elephas_amd.utils.rdd_utils import to_simple_rdd
    x, y = _data()
    sm = SparkModel(_model(), mode="synchronous", sync_granularity=gran)
    sm.fit(to_simple_rdd(SparkContext(master="local[4]"), x, y), epochs=2, batch_size=16, verbose=0,
           shuffle=False)
    for i, w in enumerate(sm.master_network.get_weights()):
        assert np.allclose(a[f"arr_{i}"], w, atol=1e-6)
    assert np.allclose(a["preds"], sm.master_network.predict(x[:50]), atol=1e-6)
    ev = sm.master_network.evaluate(x, y)
    assert np.allclose(a["ev"], ev, atol=1e-5)


@pytest.mark.parametrize("mode,ps", [("asynchronous", "socket"), ("hogwild", "http")])
def test_async_two_ranks_shared_parameter_server(tmp_path, mode, ps):
    a, b = _run(mode, ps, tmp_path)
    for k in a.files:
        if k.startswith("arr_"):
            assert np.array_equal(a[k], b[k]), k
    x, y = _data()
    assert np.isfinite(a["ev"]).all()


def _gather_rows_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    import torch.distributed as tdist
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    from elephas_amd.parallel import dist
    n = 11  # uneven blocks: 3 / 4 / 4 rows
    lo, hi = dist.block_range(n)
    local = np.arange(lo, hi, dtype=np.float32)[:, None] * np.ones((1, 5), np.float32)
    out = dist.all_gather_rows(local, n)
    np.save(os.path.join(out_dir, f"g{rank}.npy"), out)
    tdist.barrier()
    tdist.destroy_process_group()


def test_all_gather_rows_uneven_blocks(tmp_path):
    """Distributed predict's row gather (one tensor all-gather, padded blocks)."""
    port = _free_port()
    mp.start_processes(_gather_rows_worker, args=(3, port, str(tmp_path)), nprocs=3, join=True, start_method="spawn")
    want = np.arange(11, dtype=np.float32)[:, None] * np.ones((1, 5), np.float32)
    for r in range(3):
        np.testing.assert_array_equal(np.load(tmp_path / f"g{r}.npy"), want)


def _transform_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    import torch.distributed as tdist
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    from elephas_amd import config
    config.set_device("cpu")
    out = _transform_local()
    np.save(os.path.join(out_dir, f"t{rank}.npy"), out)
    tdist.barrier()
    tdist.destroy_process_group()


def _transform_local():
    from elephas_amd.data import SparkContext
    from elephas_amd.ml.adapter import to_data_frame
    from elephas_amd.ml_model import ElephasTransformer
    from elephas_amd.utils.model_utils import ModelType
    x, y = _data()
    m = _model()
    df = to_data_frame(SparkContext(master="local[4]"), x[:101], y[:101], categorical=True)
    tr = ElephasTransformer(weights=m.get_weights(), model_type=ModelType.CLASSIFICATION)
    tr.set_keras_model_config(m.to_json())
    tr.set_inference_batch_size(16)
    out = tr.transform(df)
    return np.asarray([r[tr.getOutputCol()] for r in out.collect()])


def test_transform_three_ranks_equals_single_process(tmp_path):
    """ElephasTransformer.transform splits the rows over the ranks (uneven blocks of
    101 rows), predicts each block locally and gathers them in row order: every rank
    gets exactly the single-process output (reference ml_model.py:223-242)."""
    port = _free_port()
    mp.start_processes(_transform_worker, args=(3, port, str(tmp_path)), nprocs=3, join=True, start_method="spawn")
    want = _transform_local()
    assert want.shape == (101, 3)
    for r in range(3):
        np.testing.assert_allclose(np.load(tmp_path / f"t{r}.npy"), want, rtol=0, atol=1e-6)
