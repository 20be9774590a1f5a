#!/bin/bash
mkdir -p gpurun_out
. tools/gpu_step.sh
step r5s_native 400 python -u -m pytest tests/test_native_gpu.py -q -x --timeout 200 --timeout-method thread
step r5s_gemm_check 200 python tools/gemm_check.py
step r5s_wide_w8 150 python bench.py --model wide --policy mixed_bfloat16 --steps 20 --warmup 5 --no-sub
