#!/bin/bash
mkdir -p gpurun_out
. tools/gpu_step.sh
step r5n_tests 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
step r5n_smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step r5n_bench 120 python bench.py --gpus 1 --steps 20 --warmup 5
step r5n_gemm_stamps 120 python tools/gemm_stamps.py
step r5n_gemm_check 200 python tools/gemm_check.py
