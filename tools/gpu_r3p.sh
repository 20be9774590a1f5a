#!/bin/bash
# persistent kernel clears its flags / advances counters itself (no memset / advance nodes);
# async pulls gather straight into the replica masters: GPU suite + peer tests + benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_persist_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_persist.txt 2>&1 || { echo "persist tests failed: $?"; tail -60 gpurun_out/t_persist.txt; exit 1; }
tail -2 gpurun_out/t_persist.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1 || { echo "tests failed: $?"; tail -60 gpurun_out/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/gpu_tests.txt
O=gpurun_out/r3p.log; : > $O
run() { timeout -k 10 200 python bench.py "$@" 2>/dev/null | tail -n1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*', d['ms_per_step'], round(d['value']))" >> $O; }
for i in 1 2; do
run --steps 20 --warmup 5 || exit 1
run --steps 2000 --warmup 200 || exit 1
run --mode asynchronous --frequency batch --steps 300 --warmup 30 || exit 1
run --mode hogwild --frequency batch --steps 300 --warmup 30 || exit 1
run --mode asynchronous --frequency epoch --steps 500 --warmup 50 || exit 1
done
cat $O
