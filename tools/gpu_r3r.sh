#!/bin/bash
# fp32 kind-specialised grouped GEMM variants: GPU suite + Otto / Wide / MNIST numbers + Otto stamps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1 || { echo "tests failed: $?"; tail -60 gpurun_out/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/gpu_tests.txt
O=gpurun_out/r3r.log; : > $O
run() { timeout -k 10 200 python bench.py "$@" 2>/dev/null | tail -n1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*', d['ms_per_step'], round(d['value']))" >> $O; }
for i in 1 2; do
run --model otto --batch 128 --steps 1000 --warmup 100 || exit 1
run --model wide --policy mixed_bfloat16 --workers-per-gpu 1 --batch 1024 --steps 32 --warmup 8 || exit 1
run --steps 20 --warmup 5 || exit 1
done
timeout -k 10 120 python tools/stamps.py 8 otto 128 float32 2>&1 | grep "^launch" >> $O || exit 1
cat $O
