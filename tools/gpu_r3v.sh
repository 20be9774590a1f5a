#!/bin/bash
# a layer's DW and DX on different tiles in one launch (gemm_dual): tail test, GPU suite, Otto A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_native_gpu.py -x -q --timeout 120 --timeout-method thread -k "tail_chain or throughput or one_step" > gpurun_out/t_dual.txt 2>&1 || { echo "dual tests failed: $?"; tail -60 gpurun_out/t_dual.txt; exit 1; }
tail -1 gpurun_out/t_dual.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1 || { echo "tests failed: $?"; tail -60 gpurun_out/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/gpu_tests.txt
O=gpurun_out/r3v.log; : > $O
run() { timeout -k 10 200 python bench.py "$@" 2>/dev/null | tail -n1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*', d['ms_per_step'], round(d['value']), d['config'].get('launches_per_step'))" >> $O; }
for i in 1 2; do for v in 1 0; do
ELEPHAS_AMD_DUAL=$v run --model otto --batch 128 --steps 1000 --warmup 100 || exit 1
done; done
sed -i 's/^/DUAL 1,0,1,0: /' $O
timeout -k 10 120 python tools/stamps.py 8 otto 128 float32 2>&1 | grep "^launch" >> $O || exit 1
cat $O
