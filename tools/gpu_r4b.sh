#!/bin/bash
# V2 persistent roles: persist GPU tests, headline bench (V2 and V1), stamps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_persist_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_persist.txt 2>&1; rc=$?
tail -15 gpurun_out/t_persist.txt
[ $rc -eq 0 ] || exit 1
O=gpurun_out/r4b.log; : > $O
run() { timeout -k 10 150 python bench.py "$@" 2>/dev/null | tail -n1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*', d['ms_per_step'], round(d['value']), d['config'].get('engine','')[:60])" >> $O; }
run --gpus 1 --steps 20 --warmup 5 || exit 1
run --gpus 1 --steps 2000 --warmup 50 || exit 1
ELEPHAS_AMD_PERSIST_V2=0 run --gpus 1 --steps 20 --warmup 5 || exit 1
ELEPHAS_AMD_PERSIST_V2=0 run --gpus 1 --steps 2000 --warmup 50 || exit 1
cat $O
timeout -k 10 150 python tools/persist_stamps.py 8 64 8 > gpurun_out/stamps_r4b.txt 2>&1 || exit 1
cat gpurun_out/stamps_r4b.txt | grep -v amdgpu.ids
