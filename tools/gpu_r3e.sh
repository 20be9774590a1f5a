#!/bin/bash
# big-tile variants, GPU suite, inference + async benches (partitioned persistent groups)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/big_variants.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/big_variants.txt || { echo "variants failed"; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1 || { echo "tests failed: $?"; tail -40 gpurun_out/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/gpu_tests.txt
O=gpurun_out/sweep3.jsonl; : > $O
for a in "--task predict --model wide --policy mixed_bfloat16 --steps 10 --warmup 2" "--mode asynchronous --frequency epoch --steps 500 --warmup 50" "--mode asynchronous --frequency batch --steps 300 --warmup 30" "--mode hogwild --frequency epoch --steps 500 --warmup 50" "--mode asynchronous --frequency epoch --async-groups 1 --steps 500 --warmup 50"; do
  timeout -k 10 240 python bench.py $a --out $O > gpurun_out/b.log 2>&1 || { echo "bench failed: $a"; tail -20 gpurun_out/b.log; exit 1; }
  tail -1 $O | cut -c1-150; python -c "import json;d=json.loads(open('$O').readlines()[-1]);print(d['config'].get('plan'), d['config'].get('exchange'))"
done
