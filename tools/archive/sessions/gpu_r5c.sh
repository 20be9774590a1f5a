#!/bin/bash
# round 5: GEMM kernel-only durations (rocprofv3 kernel trace of the big-tile variants and
# hipBLASLt), Otto kernel trace, Wide step
mkdir -p gpurun_out
. tools/gpu_step.sh
R=$PWD
export TMPDIR=/tmp
step r5c_gemm_stamps 120 python tools/gemm_stamps.py
step r5c_gemm_trace 240 bash -c "cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_gemm -o run -- python $R/tools/big_variants.py"
step r5c_otto_trace 180 bash -c "cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_otto -o run -- python $R/bench.py --model otto --steps 200 --warmup 20 --no-sub"
step r5c_wide 180 python bench.py --model wide --policy mixed_bfloat16 --steps 20 --warmup 5 --no-sub
