#!/bin/bash
mkdir -p gpurun_out
. tools/gpu_step.sh
step r5f_deep_tests 300 python -u -m pytest tests/test_deep_gpu.py -x -v --timeout 120 --timeout-method thread -k "not eager_exchange"
step r5f_otto 120 python bench.py --model otto --steps 200 --warmup 20 --no-sub
step r5f_deep_stamps 90 python tools/deep_stamps.py
step r5f_sync_diag3 200 python tools/sync_diag3.py
