#!/bin/bash
# Wide bf16 step with the loss rows kernel at one row per wave (LOSS_RPB 4) + kernel trace
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out
W="python $ROOT/bench.py --model wide --policy mixed_bfloat16 --workers-per-gpu 1 --batch 1024"
timeout -k 10 200 $W --steps 64 --warmup 16 > $O/wide_rpb4.log 2>&1 || exit 1
timeout -k 10 200 $W --steps 64 --warmup 16 >> $O/wide_rpb4.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/wideprof2" -o w -- $W --steps 32 --warmup 8 > "$O/wideprof2.log" 2>&1
