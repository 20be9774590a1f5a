#!/bin/bash
# DW + DX launches dispatch the deeper-tile problem first: GPU suite + A/B (Wide bf16, Otto fp32, Wide fp32-shaped MLP)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1 || { echo "tests failed: $?"; tail -60 gpurun_out/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/gpu_tests.txt
O=gpurun_out/r3t.log; : > $O
run() { timeout -k 10 200 python bench.py "$@" 2>/dev/null | tail -n1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*', d['ms_per_step'], round(d['value']))" >> $O; }
for i in 1 2; do for v in 0 1; do
ELEPHAS_AMD_NO_REORDER=$v run --model wide --policy mixed_bfloat16 --workers-per-gpu 1 --batch 1024 --steps 32 --warmup 8 || exit 1
ELEPHAS_AMD_NO_REORDER=$v run --model otto --batch 128 --steps 1000 --warmup 100 || exit 1
done; done
sed -i 's/^/NO_REORDER: /' $O
cat $O
