#!/bin/bash
# DW update epilogue: the next pass's master rows loaded ahead (rolled 256x256 passes)
mkdir -p gpurun_out
. tools/gpu_step.sh
step r5w_native_tests 400 python -u -m pytest tests/test_native_gpu.py -x -q --timeout 120 --timeout-method thread
step r5w_wide_a 150 python bench.py --model wide --policy mixed_bfloat16 --steps 20 --warmup 5 --no-sub
step r5w_wide_b 150 python bench.py --model wide --policy mixed_bfloat16 --steps 20 --warmup 5 --no-sub
step r5w_wide_stamps 240 python tools/stamps.py 8 wide 1024 mixed_bfloat16
