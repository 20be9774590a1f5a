#!/bin/bash
# V2 persistent roles, in-launch sync DP and async exchange: persist GPU tests, headline
# bench (V2 and V1), per-step sync, async batch, stamps. A failing test (rc 1) does not
# stop the run; a crash / timeout does.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_persist_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/t_persist.txt 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/t_persist.txt | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit 1; fi
O=gpurun_out/r4b.log; : > $O
run() { timeout -k 10 150 python bench.py --no-sub "$@" 2>/dev/null | tail -n1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$*', d['ms_per_step'], round(d['value']), c.get('launches_per_step'), (c.get('engine') or c.get('exchange') or '')[:70])" >> $O; }
run --gpus 1 --steps 20 --warmup 5 || exit 1
run --gpus 1 --steps 2000 --warmup 50 || exit 1
ELEPHAS_AMD_PERSIST_V2=0 run --gpus 1 --steps 20 --warmup 5 || exit 1
ELEPHAS_AMD_PERSIST_V2=0 run --gpus 1 --steps 2000 --warmup 50 || exit 1
run --gpus 1 --steps 200 --warmup 20 --granularity batch || exit 1
run --gpus 1 --steps 200 --warmup 20 --mode asynchronous --frequency batch || exit 1
run --gpus 1 --steps 200 --warmup 20 --mode hogwild --frequency batch || exit 1
cat $O
timeout -k 10 150 python tools/persist_stamps.py 8 64 8 > gpurun_out/stamps_r4b.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/stamps_r4b.txt | tail -25
