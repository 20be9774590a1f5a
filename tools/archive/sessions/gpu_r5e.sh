#!/bin/bash
# round 5: layer pipeline with 16-byte publishes + early W^T loads: tests, Otto bench + stamps
mkdir -p gpurun_out
. tools/gpu_step.sh
step r5e_deep_tests 300 python -u -m pytest tests/test_deep_gpu.py -x -v --timeout 120 --timeout-method thread
step r5e_otto 120 python bench.py --model otto --steps 200 --warmup 20 --no-sub
step r5e_deep_stamps 90 python tools/deep_stamps.py
step r5e_sync_diag2 120 python tools/sync_diag2.py
step r5e_bf16pin 90 python -u -m pytest tests/test_persist_gpu.py -x -v -s --timeout 80 --timeout-method thread -k "bf16_pinned or nobias0"
