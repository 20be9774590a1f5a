#!/bin/bash
# Wide: weight-gradient products on the 128x128 tiles (ELEPHAS_AMD_BIG_DW=0) vs the 256x256 tile, interleaved
mkdir -p gpurun_out
. tools/gpu_step.sh
step r5zx_wide_dw1_a 150 python bench.py --model wide --policy mixed_bfloat16 --steps 20 --warmup 5 --no-sub
step r5zx_wide_dw0_a 150 env ELEPHAS_AMD_BIG_DW=0 python bench.py --model wide --policy mixed_bfloat16 --steps 20 --warmup 5 --no-sub
step r5zx_wide_dw1_b 150 python bench.py --model wide --policy mixed_bfloat16 --steps 20 --warmup 5 --no-sub
step r5zx_wide_dw0_b 150 env ELEPHAS_AMD_BIG_DW=0 python bench.py --model wide --policy mixed_bfloat16 --steps 20 --warmup 5 --no-sub
