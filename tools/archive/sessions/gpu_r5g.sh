#!/bin/bash
mkdir -p gpurun_out
. tools/gpu_step.sh
step r5g_deep_tests1 300 python -u -m pytest tests/test_deep_gpu.py -x -v --timeout 120 --timeout-method thread -k "not eager_exchange"
step r5g_deep_tests2 300 python -u -m pytest tests/test_deep_gpu.py -x -v --timeout 120 --timeout-method thread -k "not eager_exchange"
step r5g_sync_diag4 200 python tools/sync_diag4.py
step r5g_otto 120 python bench.py --model otto --steps 200 --warmup 20 --no-sub
