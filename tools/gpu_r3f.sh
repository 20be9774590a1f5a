#!/bin/bash
# async groups vs hardware queue count; Wide step with the 256x256 tile for the weight gradients
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/sweep4.jsonl; : > $O
run() { timeout -k 10 240 "$@" --out $O > gpurun_out/b.log 2>&1 || { echo "bench failed: $*"; tail -20 gpurun_out/b.log; exit 1; }; tail -1 $O | cut -c1-160; }
for q in 8 16; do
  echo "== GPU_MAX_HW_QUEUES=$q"
  GPU_MAX_HW_QUEUES=$q run python bench.py --mode asynchronous --frequency epoch --steps 500 --warmup 50
  GPU_MAX_HW_QUEUES=$q run python bench.py --mode asynchronous --frequency batch --steps 300 --warmup 30
done
echo "== Wide bf16, default tiles / 256x256 tile for DW"
run python bench.py --model wide --policy mixed_bfloat16 --workers-per-gpu 1 --batch 1024 --steps 32 --warmup 8
ELEPHAS_AMD_BIG=1 run python bench.py --model wide --policy mixed_bfloat16 --workers-per-gpu 1 --batch 1024 --steps 32 --warmup 8
