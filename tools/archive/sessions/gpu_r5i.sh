#!/bin/bash
mkdir -p gpurun_out
. tools/gpu_step.sh
step r5i_deep_tests 300 python -u -m pytest tests/test_deep_gpu.py -v --timeout 120 --timeout-method thread
step r5i_otto 120 python bench.py --model otto --steps 200 --warmup 20 --no-sub
step r5i_deep_stamps 90 python tools/deep_stamps.py
step r5i_bf16pin 90 python -u -m pytest tests/test_persist_gpu.py -x -v -s --timeout 80 --timeout-method thread -k "bf16_pinned or nobias0"
