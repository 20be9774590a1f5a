#!/bin/bash
# vectorised Z accesses in the FWD / DX epilogues; batched replica-average loads
mkdir -p gpurun_out
. tools/gpu_step.sh
step r5x_native_tests 400 python -u -m pytest tests/test_native_gpu.py -x -q --timeout 120 --timeout-method thread
step r5x_wide_a 150 python bench.py --model wide --policy mixed_bfloat16 --steps 20 --warmup 5 --no-sub
step r5x_wide_b 150 python bench.py --model wide --policy mixed_bfloat16 --steps 20 --warmup 5 --no-sub
step r5x_wide_stamps 240 python tools/stamps.py 8 wide 1024 mixed_bfloat16
step r5x_host_overhead 120 python tools/host_overhead.py 20 30
step r5x_mnist_a 120 python bench.py --steps 20 --warmup 5
step r5x_mnist_b 120 python bench.py --steps 20 --warmup 5
step r5x_otto 120 python bench.py --model otto --steps 200 --warmup 20 --no-sub
