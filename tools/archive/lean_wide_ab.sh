#!/bin/bash
# Layer-0 row-major image skip on the grouped plan: Wide bf16 and Otto fp32 A/B
set -u
O=gpurun_out/lean_wide.log
W="python bench.py --model wide --policy mixed_bfloat16 --workers-per-gpu 1 --batch 1024 --steps 64 --warmup 16"
T="python bench.py --model otto --batch 128 --steps 500 --warmup 50"
for round in 1 2; do
  for v in 0 1; do
    echo "== round $round RC_LEAN=$v wide" >> $O
    ELEPHAS_AMD_RC_LEAN=$v timeout -k 10 200 $W >> $O 2>&1 || exit 1
    echo "== round $round RC_LEAN=$v otto" >> $O
    ELEPHAS_AMD_RC_LEAN=$v timeout -k 10 200 $T >> $O 2>&1 || exit 1
  done
done
