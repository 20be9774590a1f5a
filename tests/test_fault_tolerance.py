"""Failure detection: injected faults surface as exceptions in the
driver, async worker-thread failures propagate, and when one rank of a 2-rank job
dies the other one fails within the collective timeout instead of hanging."""
import os
import socket
import subprocess
import sys
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _sm(mode, **kw):
    from elephas_amd.models import Dense, Sequential
    from elephas_amd.models.optimizers import SGD
    from elephas_amd.spark_model import SparkModel
    m = Sequential([Dense(6, input_dim=4, activation="relu"), Dense(2, activation="softmax")])
    m.compile(SGD(0.1), "categorical_crossentropy")
    return SparkModel(m, mode=mode, **kw)


def _rdd(sc, n=80):
    rng = np.random.default_rng(0)
    x = rng.normal(size=(n, 4)).astype(np.float32)
    y = np.eye(2, dtype=np.float32)[rng.integers(0, 2, n)]
    return sc.parallelize(list(zip(x, y)), 2)


@pytest.mark.parametrize("phase", ["train", "allreduce"])
def test_injected_fault_fails_fast_sync(monkeypatch, spark_context, phase):
    from elephas_amd.parallel import fault
    fault.reset()
    monkeypatch.setenv("ELEPHAS_AMD_FAULT_INJECT", f"rank=0,phase={phase}")
    with pytest.raises(fault.InjectedFault):
        _sm("synchronous").fit(_rdd(spark_context), epochs=1, batch_size=8, verbose=0)


def test_async_worker_failure_propagates(monkeypatch, spark_context):
    from elephas_amd.parallel import fault
    fault.reset()
    monkeypatch.setenv("ELEPHAS_AMD_FAULT_INJECT", "rank=0,phase=push,after=1")
    sm = _sm("asynchronous", parameter_server_mode="socket", port=23411)
    with pytest.raises(fault.InjectedFault):
        sm.fit(_rdd(spark_context), epochs=3, batch_size=8, verbose=0)
    sm.stop_server()


def test_fault_spec_parsing(monkeypatch):
    from elephas_amd.parallel import fault
    fault.reset()
    monkeypatch.setenv("ELEPHAS_AMD_FAULT_INJECT", "rank=1,phase=pull,after=2")
    fault.maybe_inject("pull", 0)          # other rank: no-op
    fault.maybe_inject("train", 1)         # other phase: no-op
    fault.maybe_inject("pull", 1)
    fault.maybe_inject("pull", 1)
    with pytest.raises(fault.InjectedFault):
        fault.maybe_inject("pull", 1)


_SCRIPT = r'''
import os, sys, numpy as np
sys.path.insert(0, {root!r})
from elephas_amd import config
config.set_device("cpu")
from elephas_amd.data import SparkContext
from elephas_amd.models import Dense, Sequential
from elephas_amd.models.optimizers import SGD
from elephas_amd.spark_model import SparkModel
m = Sequential([Dense(6, input_dim=4, activation="relu"), Dense(2, activation="softmax")])
m.compile(SGD(0.1), "categorical_crossentropy")
sm = SparkModel(m, mode="synchronous")
rng = np.random.default_rng(0)
x = rng.normal(size=(80, 4)).astype(np.float32)
y = np.eye(2, dtype=np.float32)[rng.integers(0, 2, 80)]
sm.fit(SparkContext(master="local[4]").parallelize(list(zip(x, y)), 4), epochs=1, batch_size=8, verbose=0)
print("finished", flush=True)
'''


def test_peer_failure_does_not_hang(tmp_path):
    """Rank 1 dies before the all-reduce; rank 0 must error out within the
    collective timeout (gloo here; RCCL uses the same timeout + async error handling)."""
    script = tmp_path / "job.py"
    script.write_text(_SCRIPT.format(root=ROOT))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, ELEPHAS_AMD_FAULT_INJECT="rank=1,phase=allreduce", ELEPHAS_AMD_COLLECTIVE_TIMEOUT="20",
               CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", PYTHONPATH=ROOT)
    t0 = time.time()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr=127.0.0.1", f"--master-port={port}", str(script)],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode != 0
    assert "finished" not in r.stdout
    assert "InjectedFault" in r.stderr
    assert time.time() - t0 < 200
