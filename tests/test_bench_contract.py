"""bench.py's driver contract on the CPU (gloo, torch reference engine): ONE JSON line
from rank 0 with the BASELINE.json metric, the whole-job aggregate, n_gpus == world
size, for both launch forms the driver uses -- ``bench.py --gpus N`` (bench spawns
its own ranks) and ``torch.distributed.run ... bench.py --gpus N``."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _json_lines(out: str):
    lines = []
    for ln in out.splitlines():
        ln = ln.strip()
        if ln.startswith("{") and ln.endswith("}"):
            lines.append(json.loads(ln))
    return lines


def _check(rec, n):
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        baseline = json.load(f)
    assert KEYS <= set(rec), KEYS - set(rec)
    assert rec["metric"] == baseline["metric"]
    assert rec["n_gpus"] == n and rec["config"]["ranks"] == n
    assert rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["value"] > 0 and rec["higher_is_better"] is True
    assert rec["dtype"] == "fp32" and rec["scaling"] in ("weak", "strong")
    # whole-job aggregate: samples of every worker of every rank over the timed steps
    cfg = rec["config"]
    per_step = cfg["workers_total"] * cfg["batch_per_worker"]
    assert abs(rec["value"] * rec["ms_per_step"] / 1e3 - per_step) / per_step < 0.05


def _env():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    env["MASTER_ADDR"] = "127.0.0.1"
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    return env


@pytest.mark.parametrize("n", [1, 2])
def test_bench_self_spawn_prints_one_json_line(n):
    env = _env()
    env["MASTER_PORT"] = str(_free_port())
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(n), "--steps", "2", "--warmup", "1"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout[-2000:]
    _check(recs[0], n)


def test_bench_under_torchrun_prints_one_json_line():
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
                        "--steps", "2", "--warmup", "1"], cwd=ROOT, env=_env(), capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout[-2000:]
    _check(recs[0], 2)


def test_bench_deadline_prints_line_when_a_rank_stalls():
    """Job-wide deadline: rank 1 hangs at the start of the per-step-sync sub-measurement
    (fault injection, stall=1), so rank 0 blocks in that measurement's first collective.
    The headline line must still appear -- within the deadline, with every pending
    sub-measurement marked {"error": "deadline"} -- and the job must end."""
    import time
    env = _env()
    env["MASTER_PORT"] = str(_free_port())
    env["ELEPHAS_AMD_BENCH_DEADLINE_S"] = "45"
    env["ELEPHAS_AMD_FAULT_INJECT"] = "rank=1,phase=bench_sub:per_step_sync,stall=1"
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=300)
    elapsed = time.monotonic() - t0
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, (r.stdout[-2000:], r.stderr[-2000:])
    _check(recs[0], 2)
    subs = recs[0]["config"]["sub_measurements"]
    assert subs["per_step_sync"] == {"error": "deadline"}, subs
    assert subs["strong"] == {"error": "deadline"}, subs
    assert recs[0]["deadline_s"] == 45
    assert "deadline" in r.stderr
    assert elapsed < 45 + 60, elapsed   # the deadline (+ process teardown), not the collective timeout
