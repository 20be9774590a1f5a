#!/bin/bash
# round 5: layer pipeline with acquire + plain loads: tests, Otto bench + stamps, sync diagnostic
mkdir -p gpurun_out
. tools/gpu_step.sh
step r5d_deep_tests 300 python -u -m pytest tests/test_deep_gpu.py -x -v --timeout 120 --timeout-method thread -k "not eager_exchange"
step r5d_otto 120 python bench.py --model otto --steps 200 --warmup 20 --no-sub
step r5d_deep_stamps 90 python tools/deep_stamps.py
step r5d_sync_diag 120 python tools/sync_diag.py
step r5d_mnist_deep 90 env ELEPHAS_AMD_DEEP=2 python bench.py --steps 200 --warmup 20 --no-sub
step r5d_deep_sync_tests 200 python -u -m pytest tests/test_deep_gpu.py -v --timeout 120 --timeout-method thread -k "eager_exchange"
step r5d_bf16pin 90 python -u -m pytest tests/test_persist_gpu.py -x -v -s --timeout 80 --timeout-method thread -k "bf16_pinned or nobias0"
