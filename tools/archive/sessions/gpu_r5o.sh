#!/bin/bash
# Wide-MLP bf16: default plan vs the 256x256 tile (ELEPHAS_AMD_BIG=1), kernel trace of both
mkdir -p gpurun_out
. tools/gpu_step.sh
R=$PWD
export TMPDIR=/tmp
step r5o_wide 150 python bench.py --model wide --policy mixed_bfloat16 --steps 20 --warmup 5 --no-sub
step r5o_wide_big 150 env ELEPHAS_AMD_BIG=1 python bench.py --model wide --policy mixed_bfloat16 --steps 20 --warmup 5 --no-sub
step r5o_wide_trace 240 bash -c "cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_wide -o run -- python $R/bench.py --model wide --policy mixed_bfloat16 --steps 20 --warmup 5 --no-sub"
step r5o_wide_big_trace 240 bash -c "cd /tmp && ELEPHAS_AMD_BIG=1 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_wide_big -o run -- python $R/bench.py --model wide --policy mixed_bfloat16 --steps 20 --warmup 5 --no-sub"
