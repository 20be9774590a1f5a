#!/bin/bash
# async frequency='batch': persistent groups pull straight into P (no image refresh) vs row-chain groups
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_peer_gpu.py -x -q --timeout 300 --timeout-method thread -k "async or ps" > gpurun_out/t_async.txt 2>&1 || { echo "tests failed: $?"; tail -60 gpurun_out/t_async.txt; exit 1; }
tail -2 gpurun_out/t_async.txt
timeout -k 10 300 python -u -m pytest tests/test_native_gpu.py -x -q --timeout 120 --timeout-method thread -k "spark_model or ps_" > gpurun_out/t_async2.txt 2>&1 || { echo "tests failed: $?"; tail -60 gpurun_out/t_async2.txt; exit 1; }
tail -2 gpurun_out/t_async2.txt
O=gpurun_out/r3n.log; : > $O
run() { timeout -k 10 200 python bench.py "$@" 2>/dev/null | tail -n1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*', d['ms_per_step'], round(d['value']))" >> $O; }
for i in 1 2; do
run --mode asynchronous --frequency batch --steps 300 --warmup 30 || exit 1
ELEPHAS_AMD_PERSIST=0 run --mode asynchronous --frequency batch --steps 300 --warmup 30 || exit 1
run --mode hogwild --frequency batch --steps 300 --warmup 30 || exit 1
run --mode asynchronous --frequency epoch --steps 500 --warmup 50 || exit 1
done
cat $O
