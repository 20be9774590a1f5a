#!/usr/bin/env python
"""One parameterised GPU session driver (run on an MI355X box through gpurun):

    gpurun -- python tools/gpu.py STEP [STEP ...]

Every step runs under its own time limit with its output in gpurun_out/<tag>.txt; a step
that hangs or crashes (time limit, abort, segfault) ends the session -- nothing else
touches the GPU after it.  Steps (arguments are comma-separated, no spaces):

  tests[:EXPR]            pytest -m gpu over tests/ (-k EXPR)
  file:PATH[:EXPR]        pytest over one test file (-k EXPR)
  smoke                   __graft_entry__.smoke()
  bench:ARGS              bench.py ARGS, the JSON line appended to gpurun_out/session.jsonl
  ab:VAR=V1|V2:ARGS       bench.py ARGS with $VAR = V1, V2, V1, V2 (A/B in one box)
  prof:NAME:ARGS          rocprofv3 --kernel-trace --stats of bench.py ARGS -> gpurun_out/prof_NAME
  pmc:NAME:CTRS:ARGS      one rocprofv3 --pmc pass (CTRS '+'-separated, within one pass's limits)
  py:SCRIPT[:ARGS]        python tools/SCRIPT ARGS (stamps.py, persist_stamps.py, gemm_check.py, ...)
  micro:NAME              hipcc tools/micro/NAME.hip for gfx950 and run it (120 s limit)

Any step may carry a tag and environment overrides in front of it:

  [TAG/][VAR=VAL[+VAR=VAL...]@]STEP
  e.g.  sync_rs/ELEPHAS_AMD_XCHG_RS=1@py:persist_stamps.py:8,64,8,-1,float32,sync

(output in gpurun_out/TAG.txt).  The profiles under profiles/ name the step that produced
them (profiles/README.md); tools/archive/sessions/ keeps the earlier one-file session scripts that
produced the older ones.
"""
from __future__ import annotations

import json
import os
import signal
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
FATAL = {124, 137, 134, 139, -6, -9, -11}


def _run(tag: str, cmd, timeout: int, env=None, cwd=None) -> int:
    path = os.path.join(OUT, tag + ".txt")
    print(f"== {tag}: {' '.join(cmd)}", flush=True)
    t0 = time.time()
    with open(path, "w") as f:
        p = subprocess.Popen(cmd, stdout=f, stderr=subprocess.STDOUT, env=env, cwd=cwd or ROOT,
                             start_new_session=True)
        try:
            rc = p.wait(timeout=timeout)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGTERM)
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
            rc = 124
    with open(path) as f:
        tail = f.read().splitlines()[-3:]
    print(f"   rc={rc} {time.time() - t0:.1f}s", *("   | " + t[:300] for t in tail), sep="\n", flush=True)
    return rc


def _bench(args, env=None, tag="bench"):
    out = os.path.join(OUT, "session.jsonl")
    return _run(tag, [sys.executable, "bench.py"] + args + ["--out", out], 300, env=env)


def parse_step(step: str, n: int):
    """'[TAG/][VAR=VAL[+VAR=VAL...]@]KIND[:REST]' -> (tag, env overrides, kind, rest)."""
    tag = None
    head, sep, tail = step.partition("@")
    if sep and "=" in head:
        envspec, step = head, tail
    else:
        envspec = ""
    if "/" in envspec.split("=")[0]:
        tag, _, envspec = envspec.partition("/")
    elif not envspec and "/" in step.split(":")[0]:
        tag, _, step = step.partition("/")
    env = dict(kv.split("=", 1) for kv in envspec.split("+")) if envspec else {}
    kind, _, rest = step.partition(":")
    return tag or f"s{n:02d}_{kind}", env, kind, rest


def main(steps):
    os.makedirs(OUT, exist_ok=True)
    n = 0
    for step in steps:
        n += 1
        tag, extra, kind, rest = parse_step(step, n)
        saved = {k: os.environ.get(k) for k in extra}
        os.environ.update(extra)   # inherited by this step's child (restored below)
        if kind == "tests":
            cmd = [sys.executable, "-u", "-m", "pytest", "tests", "-m", "gpu", "-x", "-q", "--timeout", "300",
                   "--timeout-method", "thread"] + (["-k", rest] if rest else [])
            rc = _run(tag, cmd, 1500)
        elif kind == "file":
            path, _, expr = rest.partition(":")
            cmd = [sys.executable, "-u", "-m", "pytest", path, "-x", "-v", "--timeout", "300",
                   "--timeout-method", "thread"] + (["-k", expr] if expr else [])
            rc = _run(tag, cmd, 900)
        elif kind == "smoke":
            rc = _run(tag, [sys.executable, "-c", "import __graft_entry__ as g; g.smoke()"], 300)
        elif kind == "bench":
            rc = _bench(rest.split(",") if rest else [], tag=tag)
        elif kind == "ab":
            var, _, tail = rest.partition(":")
            name, _, vals = var.partition("=")
            a, b = vals.split("|")
            rc = 0
            for i, v in enumerate((a, b, a, b)):
                rc = _bench(tail.split(",") if tail else [], env=dict(os.environ, **{name: v}),
                            tag=f"{tag}_{name}_{v}_{i}")
                if rc in FATAL:
                    break
        elif kind == "prof":
            name, _, tail = rest.partition(":")
            d = os.path.join(OUT, "prof_" + name)
            cmd = ["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", d, "-o", "run", "--",
                   sys.executable, os.path.join(ROOT, "bench.py")] + (tail.split(",") if tail else [])
            rc = _run(tag, cmd, 600, env=dict(os.environ, TMPDIR="/tmp"), cwd="/tmp")
        elif kind == "pmc":
            name, _, tail = rest.partition(":")
            ctrs, _, args = tail.partition(":")
            d = os.path.join(OUT, "pmc_" + name)
            cmd = ["rocprofv3", "--pmc"] + ctrs.split("+") + ["--output-format", "csv", "-d", d, "-o", "p", "--",
                                                            sys.executable, os.path.join(ROOT, "bench.py")]
            cmd += args.split(",") if args else []
            rc = _run(tag, cmd, 120, env=dict(os.environ, TMPDIR="/tmp"), cwd="/tmp")
        elif kind == "micro":
            exe = os.path.join("/tmp", "micro_" + rest)
            rc = _run(tag + "_build", ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                                       os.path.join(ROOT, "tools", "micro", rest + ".hip"), "-o", exe], 300)
            if rc == 0:
                rc = _run(tag, [exe], 120)
        elif kind == "py":
            script, _, args = rest.partition(":")
            rc = _run(tag, [sys.executable, os.path.join("tools", script)] + (args.split(",") if args else []), 600)
        else:
            raise SystemExit(f"unknown step {step!r}")
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        if rc in FATAL:
            print(f"stopping: {step} ended with {rc}", flush=True)
            return rc
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
