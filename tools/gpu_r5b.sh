#!/bin/bash
# round 5: layer-pipeline kernel tests, Otto bench, GPU suite
mkdir -p gpurun_out
. tools/gpu_step.sh
step r5b_deep_tests 600 python -u -m pytest tests/test_deep_gpu.py -x -v --timeout 120 --timeout-method thread
step r5b_otto 180 python bench.py --model otto --steps 200 --warmup 20 --no-sub
step r5b_otto_tail 180 env ELEPHAS_AMD_DEEP=0 python bench.py --model otto --steps 200 --warmup 20 --no-sub
step r5b_mnist 120 python bench.py --steps 20 --warmup 5
