#!/bin/bash
# round 5: layer-pipeline kernel tests, Otto bench, fit benches, bf16 pin
mkdir -p gpurun_out
. tools/gpu_step.sh
step r5b_deep_tests 420 python -u -m pytest tests/test_deep_gpu.py -x -v --timeout 120 --timeout-method thread
step r5b_otto 120 python bench.py --model otto --steps 200 --warmup 20 --no-sub
step r5b_deep_stamps 90 python tools/deep_stamps.py
step r5b_mnist_deep 90 env ELEPHAS_AMD_DEEP=2 python bench.py --steps 200 --warmup 20 --no-sub
step r5b_mnist_deep_sync 90 env ELEPHAS_AMD_DEEP=2 python bench.py --granularity batch --steps 200 --warmup 20 --no-sub
step r5b_bf16pin 90 python -u -m pytest tests/test_persist_gpu.py -x -v -s --timeout 80 --timeout-method thread -k "bf16_pinned or nobias0"
step r5b_otto_fit 120 python bench.py --model otto --task fit --steps 5 --warmup 2
step r5b_mnist 90 python bench.py --steps 20 --warmup 5
