#!/bin/bash
# SparkModel.fit wall benchmark (weak + strong), the full Otto notebook config, and a
# kernel trace of the 1-worker step (the per-GPU shape of the strong 8-GPU config).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --task fit --steps 3 --warmup 1 > $OUT/fit.log 2>&1 || exit $?
tail -1 $OUT/fit.log | cut -c1-1200
timeout -k 10 300 python bench.py --task fit --steps 3 --warmup 1 --scaling strong > $OUT/fit_strong.log 2>&1 || exit $?
tail -1 $OUT/fit_strong.log | cut -c1-1200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_w1 -o w1 -- python bench.py --steps 300 --warmup 30 --workers-per-gpu 1 > $OUT/prof_w1.log 2>&1 || exit $?
python tools/trace_steps.py $OUT/prof_w1/w1_kernel_trace.csv 600 2>&1 | head -6
timeout -k 10 400 python tools/otto_full.py > $OUT/otto_full.log 2>&1 || exit $?
tail -1 $OUT/otto_full.log
