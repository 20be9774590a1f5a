"""Multi-process GPU tests of the peer-memory paths (csrc/kernels/peer.hip):
two ranks (processes) share the one MI355X of the test box and map each other's
buffers through HIP IPC, exactly as ranks on different GPUs of a node do over xGMI.
Each scenario runs tests/_peer_worker.py once per rank under a gloo process group."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _run(scenario, world=2, timeout=150, env_extra=None):
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(world):
        # the ranks share the GPU: parallel/dist.py detects it (device UUIDs) and sizes
        # every persistent grid to an equal CU share, so both stay resident
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        env.update(env_extra or {})
        cmd = [sys.executable, "-u", os.path.join(HERE, "_peer_worker.py"), scenario]
        prof = os.environ.get("ELEPHAS_AMD_PEER_PROF_DIR")   # tools: kernel trace of rank 0
        if prof and r == 0:
            cmd = ["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", prof, "-o",
                   scenario, "--"] + cmd
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=timeout)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    res = []
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out[-3000:]
        line = [ln for ln in out.splitlines() if ln.startswith("RESULT ")]
        assert line, out[-3000:]
        res.append(json.loads(line[-1][7:]))
    return sorted(res, key=lambda d: d["rank"])


def test_peer_allreduce_two_processes():
    """One-shot, two-shot and auto selection over sizes from 1 element to more than the
    staging capacity (chunked calls) and odd tails: every rank's result equals the fp32
    rank-order sum bit for bit, and all ranks agree; a misaligned view works too."""
    for r in _run("allreduce"):
        assert r["self_test"] and r["error"] == 0 and r["misaligned_ok"], r
        assert r["barrier_waited"] >= 0.25, r     # the peer barrier waited for the late rank
        bad = [c for c in r["cases"] if not (c["exact"] and c["same_on_all_ranks"])]
        assert not bad, bad


def test_per_step_allreduce_in_graph_matches_eager_gloo():
    """The per-step DP path with the peer all-reduce captured inside the step's hipGraph
    (16 steps per replay, device-side call epochs) gives bit-identical weights to the
    eager path that all-reduces the same gradients through gloo, on both ranks."""
    for r in _run("step_graph"):
        assert r["error"] == 0 and r["same_on_all_ranks"] and r["moved"] > 0, r
        assert r["bit_equal"], r


def test_sharded_ps_two_processes():
    """Sharded device PS over two processes: concurrent pushes from both ranks are all
    applied (integer deltas, exact), asynchronous pulls never see a torn chunk."""
    res = _run("ps")
    for r in res:
        assert r["final_exact"] and r["torn_chunks"] == 0 and r["error"] == 0, r
    assert res[0]["shard_begin"][0] == 0 and res[0]["shard_begin"][1] > 0


@pytest.mark.parametrize("mode", ["asynchronous", "hogwild"])
def test_spark_model_async_two_ranks_learns(mode):
    """SparkModel asynchronous / hogwild (frequency='batch') with two ranks, each with two
    independently progressing worker groups, on the sharded device PS: the master
    network learns a learnable synthetic task and ends identical on both ranks."""
    for r in _run(f"spark_{mode}"):
        assert r["finite"] and r["same_on_all_ranks"], r
        assert r["acc"] > max(0.6, r["acc0"] + 0.3), r


def test_ps_self_test_passes_and_catches_a_bad_rank():
    """DeviceClient.connect runs a voted self-test of the sharded PS (concurrent exact
    integer pushes, torn-chunk check in asynchronous mode); a rank that contributes a
    wrong delta makes every rank raise instead of training on a broken server."""
    for r in _run("ps_selftest"):
        for mode in ("asynchronous", "hogwild"):
            v = r[mode]
            assert not v["raised"], v
            assert all(x["exact"] and x["error"] == 0 and x["torn_chunks"] == 0 for x in v["votes"]), v
    for r in _run("ps_selftest", env_extra={"ELEPHAS_AMD_FAULT_INJECT": "rank=1,phase=ps_selftest"}):
        assert r["asynchronous"]["raised"] and "self-test failed" in r["asynchronous"]["msg"], r


@pytest.mark.parametrize("gran", ["fit", "epoch", "batch"])
def test_spark_model_synchronous_two_ranks_equals_single_process(tmp_path, gran):
    """SparkModel(mode='synchronous') with two ranks on the native engine, averaging /
    gradient exchange through the peer all-reduce (reference integration matrix,
    tests/integration/test_end_to_end.py:18-67 with num_workers=2), then distributed
    predict, evaluate and ElephasTransformer.transform: both ranks agree bit for bit and
    match a single-process run over the same 4 partitions."""
    env = {"ELEPHAS_AMD_TEST_OUT": str(tmp_path), "ELEPHAS_AMD_P2P_ANY_BACKEND": "1"}
    two = _run(f"spark_sync_{gran}", env_extra=env)
    one = _run(f"spark_sync_{gran}", world=1, env_extra=env)
    for r in two:
        assert r["peer_path"] and r["same_on_all_ranks"] and r["native"] and r["histories"] == 4, r
    a, b = (np.load(tmp_path / f"{gran}_w2_r{r}.npz") for r in (0, 1))
    ref = np.load(tmp_path / f"{gran}_w1_r0.npz")
    for k in a.files:
        assert np.array_equal(a[k], b[k]), k
    for k in a.files:
        scale = max(1.0, float(np.abs(ref[k]).max()))
        np.testing.assert_allclose(a[k], ref[k], rtol=0, atol=2e-6 * scale, err_msg=k)


@pytest.mark.parametrize("gran", ["fit", "epoch"])
def test_spark_model_sync_persistent_plan_two_ranks_match_one(gran, tmp_path):
    """The persistent plan under SparkModel(mode='synchronous') across 2 ranks (each rank's
    persistent grid sized to half the CUs by the device-sharing detection, so both stay
    resident on the shared GPU):
    the averaging writes the mean into the masters and leaves the weight images to the
    next reader (NativeTrainer._ensure_images) -- both ranks agree bit for bit and match a
    single-process run; predict / evaluate / transform read refreshed images."""
    env = {"ELEPHAS_AMD_TEST_OUT": str(tmp_path), "ELEPHAS_AMD_P2P_ANY_BACKEND": "1",
           "ELEPHAS_AMD_PERSIST": "1"}
    two = _run(f"spark_sync_{gran}p", env_extra=env)
    one = _run(f"spark_sync_{gran}p", world=1, env_extra=env)
    for r in two + one:
        assert r["persistent"] and r["same_on_all_ranks"] and r["native"] and r["histories"] == 4, r
    for r in two:
        assert r["peer_path"], r
    a, b = (np.load(tmp_path / f"{gran}p_w2_r{r}.npz") for r in (0, 1))
    ref = np.load(tmp_path / f"{gran}p_w1_r0.npz")
    for k in a.files:
        assert np.array_equal(a[k], b[k]), k
    for k in a.files:
        scale = max(1.0, float(np.abs(ref[k]).max()))
        np.testing.assert_allclose(a[k], ref[k], rtol=0, atol=2e-6 * scale, err_msg=k)


def test_sync_inlaunch_across_ranks_matches_one_model():
    """Per-step synchronous DP across ranks inside the persistent launch (the replica sum
    of every weight-gradient tile exchanged with the other rank through peer-mapped
    buffers, summed in rank order): all replicas of both ranks stay bit-identical and
    match one fp32 torch model trained on the stacked batches of the 2 x 2 workers."""
    for r in _run("sync_inlaunch"):
        assert r["attached"], r
        assert r["error"] == 0 and r["replicas_equal"] and r["same_on_all_ranks"], r
        assert r["err"] < 1e-3, r
        # 2 epochs x 9 steps ran with the exchange, after the 2 steps of the attach's self-test
        assert r["steps_tagged"] == 18 + 2, r


def test_rank_exchange_selftest_votes_and_falls_back():
    """The in-launch rank exchange is trusted only after a voted numeric self-test (known
    integer tiles through its own buffers, flags and tags, checked against the exact rank
    sums): clean -> every rank attaches and trains inside the launch; a rank that sends a
    wrong tile (fault injection) -> every rank detaches, and the per-step all-reduce
    fallback still trains to the single-model result on both ranks."""
    for r in _run("xrank_selftest"):
        assert r["attached"] and r["selftest"]["ok"], r
        assert all(v == [0, 0] for v in r["selftest"]["votes"]), r
        assert r["same_on_all_ranks"] and r["err"] < 1e-3, r
    for r in _run("xrank_selftest", env_extra={"ELEPHAS_AMD_FAULT_INJECT": "rank=1,phase=xrank_selftest"}):
        assert not r["attached"] and r["selftest"] is not None and not r["selftest"]["ok"], r
        assert any(v[0] > 0 for v in r["selftest"]["votes"]), r
        assert r["same_on_all_ranks"] and r["err"] < 1e-3, r


def test_sync_inlaunch_across_ranks_layer_pipeline_matches_one_model():
    """The layer pipeline's rank exchange (deep_impl.h exchange: the replicas' reduce-scatter
    of every gradient tile, each slice then summed over the ranks through peer-mapped
    buffers in rank order): an Otto-like 93-256-256-9 stack, 2 ranks x 2 replicas, stays
    bit-identical on every replica of every rank and matches ONE fp32 torch model trained
    on the four workers' stacked batches."""
    for r in _run("sync_inlaunch_deep"):
        assert r["attached"], r
        assert "layer pipeline" in r["plan"], r
        assert r["error"] == 0 and r["replicas_equal"] and r["same_on_all_ranks"], r
        assert r["err"] < 1e-3, r
        assert r["steps_tagged"] == 18 + 2, r


def test_rank_exchange_selftest_layer_pipeline_votes_and_falls_back():
    """The layer pipeline's rank exchange is voted in by its own numeric self-test
    (deep_xrank_selftest_kernel: known integer slices through the same buffers, flags and
    tags): clean -> attached and trained inside the launch; a corrupting rank (fault
    injection phase=xrank_selftest) -> every rank detaches and the per-step all-reduce
    fallback still reaches the one-model result."""
    for r in _run("xrank_selftest_deep"):
        assert r["attached"] and r["selftest"]["ok"], r
        assert r["same_on_all_ranks"] and r["err"] < 1e-3, r
    for r in _run("xrank_selftest_deep", env_extra={"ELEPHAS_AMD_FAULT_INJECT": "rank=1,phase=xrank_selftest"}):
        assert not r["attached"] and not r["selftest"]["ok"], r
        assert any(v[0] > 0 for v in r["selftest"]["votes"]), r
        assert r["same_on_all_ranks"] and r["err"] < 1e-3, r
