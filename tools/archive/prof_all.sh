#!/bin/bash
# Kernel-trace + stats summaries of the benchmark configs (copied to profiles/ by hand).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$name" -o k -- "$@" > "$OUT/$name.log" 2>&1 || return $?; }
run p_mnist python "$ROOT/bench.py" --steps 300 --warmup 30 || exit $?
run p_otto python "$ROOT/bench.py" --model otto --batch 128 --steps 200 --warmup 20 || exit $?
run p_wide python "$ROOT/bench.py" --model wide --workers-per-gpu 1 --batch 1024 --steps 20 --warmup 3 || exit $?
