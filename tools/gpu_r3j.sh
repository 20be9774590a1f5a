#!/bin/bash
# tail-chain plan (Otto) + lazy image refresh: GPU suite, Otto A/B tail on/off, stamps, driver shape
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_native_gpu.py -x -q --timeout 120 --timeout-method thread -k tail_chain > gpurun_out/t_tail.txt 2>&1 || { echo "tail tests failed: $?"; tail -60 gpurun_out/t_tail.txt; exit 1; }
tail -2 gpurun_out/t_tail.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1 || { echo "tests failed: $?"; tail -60 gpurun_out/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/gpu_tests.txt
O=gpurun_out/r3j.log; : > $O
for round in 1 2; do for v in -1 0; do
  ELEPHAS_AMD_TAIL=$v timeout -k 10 200 python bench.py --model otto --batch 128 --steps 1000 --warmup 100 2>/dev/null | tail -n1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$round TAIL=$v otto', d['ms_per_step'], d['config'].get('launches_per_step'))" >> $O || exit 1
done; done
for i in 1 2; do timeout -k 10 120 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -n1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('driver shape', d['ms_per_step'], round(d['value']))" >> $O || exit 1; done
timeout -k 10 120 python tools/stamps.py 8 otto 128 float32 2>&1 | grep "^launch" >> $O || exit 1
cat $O
