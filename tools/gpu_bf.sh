#!/bin/bash
# bf16 persistent instance: its GPU tests and the bench, fp32 and bf16 side by side
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_persist_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/t_bf.txt 2>&1; rc=$?
tail -3 gpurun_out/t_bf.txt; grep -E "FAILED|rel " gpurun_out/t_bf.txt | head
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit 1
O=gpurun_out/bf.log; : > $O
run() { timeout -k 10 150 python bench.py --no-sub "$@" 2>/dev/null | tail -n1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*', d['dtype'], d['ms_per_step'], round(d['value']))" >> $O; }
for p in float32 mixed_bfloat16; do
  run --policy $p --steps 20 --warmup 5 || exit 1
  run --policy $p --steps 2000 --warmup 50 || exit 1
done
cat $O
timeout -k 10 150 python tools/persist_stamps.py 8 64 8 -1 mixed_bfloat16 > gpurun_out/stamps_bf.txt 2>&1 || exit 1
grep -E "step 5|period" gpurun_out/stamps_bf.txt
