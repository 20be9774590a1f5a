#!/bin/bash
# round 5 baseline: GPU suite, default bench, Otto bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5a_tests.txt 2>&1 || { echo "tests failed: $?"; tail -30 gpurun_out/r5a_tests.txt; exit 1; }
tail -3 gpurun_out/r5a_tests.txt
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/r5a_bench.txt 2>&1 && tail -1 gpurun_out/r5a_bench.txt
timeout -k 10 120 python bench.py --model otto --steps 200 --warmup 20 --no-sub > gpurun_out/r5a_otto.txt 2>&1 && tail -1 gpurun_out/r5a_otto.txt
