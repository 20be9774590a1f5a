#!/bin/bash
# Wide-MLP bf16 step (1 worker x 1024): DW/DX launch split A/B, two rounds, + kernel trace
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/wide_ab.log
W="python $ROOT/bench.py --model wide --policy mixed_bfloat16 --workers-per-gpu 1 --batch 1024 --steps 64 --warmup 16"
for round in 1 2; do
  for s in 0 1; do
    echo "== round $round ELEPHAS_AMD_SPLIT_DWDX=$s" >> $O
    ELEPHAS_AMD_SPLIT_DWDX=$s timeout -k 10 200 $W >> $O 2>&1 || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
ELEPHAS_AMD_SPLIT_DWDX=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/wideprof" -o w -- python "$ROOT/bench.py" --model wide --policy mixed_bfloat16 --workers-per-gpu 1 --batch 1024 --steps 32 --warmup 8 > "$ROOT/gpurun_out/wideprof.log" 2>&1
