#!/bin/bash
# full GPU suite + smoke + headline bench + Otto fit + GEMM stamps (round-5 checkpoint)
mkdir -p gpurun_out
. tools/gpu_step.sh
step r5j_tests 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
step r5j_smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step r5j_bench 120 python bench.py
step r5j_otto_fit 120 python bench.py --model otto --task fit --steps 5 --warmup 2
step r5j_mnist_fit 120 python bench.py --task fit --steps 5 --warmup 2
step r5j_gemm_stamps 120 python tools/gemm_stamps.py
