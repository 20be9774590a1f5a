#!/bin/bash
# Wide-MLP bf16 tile choice: 1 and 8 workers per GPU, THR vs the 256x256 tile
mkdir -p gpurun_out
. tools/gpu_step.sh
step r5p_w1 120 python bench.py --model wide --policy mixed_bfloat16 --workers-per-gpu 1 --steps 20 --warmup 5 --no-sub
step r5p_w1_big 120 env ELEPHAS_AMD_BIG=1 python bench.py --model wide --policy mixed_bfloat16 --workers-per-gpu 1 --steps 20 --warmup 5 --no-sub
step r5p_w8 150 python bench.py --model wide --policy mixed_bfloat16 --steps 20 --warmup 5 --no-sub
step r5p_w8_big 150 env ELEPHAS_AMD_BIG=1 python bench.py --model wide --policy mixed_bfloat16 --steps 20 --warmup 5 --no-sub
step r5p_w1_big_b 120 env ELEPHAS_AMD_BIG=1 python bench.py --model wide --policy mixed_bfloat16 --workers-per-gpu 1 --steps 20 --warmup 5 --no-sub
step r5p_w1_b 120 python bench.py --model wide --policy mixed_bfloat16 --workers-per-gpu 1 --steps 20 --warmup 5 --no-sub
