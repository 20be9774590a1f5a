#!/bin/bash
# XCD-grouped tile order of single-problem grouped launches: plain GEMM + Wide step A/B
set -u
O=gpurun_out/xcd_ab.log
W="python bench.py --model wide --policy mixed_bfloat16 --workers-per-gpu 1 --batch 1024 --steps 64 --warmup 16"
for round in 1 2; do
  for v in 0 1; do
    echo "== round $round XCD_ORDER=$v" >> $O
    ELEPHAS_AMD_XCD_ORDER=$v timeout -k 10 120 python tools/gemm_check.py >> $O 2>&1 || exit 1
    ELEPHAS_AMD_XCD_ORDER=$v timeout -k 10 200 $W >> $O 2>&1 || exit 1
  done
done
