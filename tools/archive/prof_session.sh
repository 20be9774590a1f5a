#!/bin/bash
# rocprofv3 kernel-trace sessions for diagnostics
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$name" -o k -- "$@" > "$OUT/$name.log" 2>&1; echo "$name rc=$?"; }
run prof_kbench python "$ROOT/tools/kernel_bench.py" || exit 1
run prof_nodrop python "$ROOT/bench.py" --steps 200 --warmup 20 --dropout 0 || exit 1
run prof_w1 python "$ROOT/bench.py" --steps 200 --warmup 20 --workers-per-gpu 1 || exit 1
