#!/bin/bash
mkdir -p gpurun_out
. tools/gpu_step.sh
step r5h_grad_diag 120 python tools/grad_diag.py 2
step r5h_deep_tests 300 python -u -m pytest tests/test_deep_gpu.py -v --timeout 120 --timeout-method thread -k "not eager_exchange"
step r5h_otto 120 python bench.py --model otto --steps 200 --warmup 20 --no-sub
step r5h_deep_stamps 90 python tools/deep_stamps.py
