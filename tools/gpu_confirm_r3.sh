#!/bin/bash
# end-of-session confirmation of the committed build: GPU suite, smoke, default bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1 || { echo "tests failed: $?"; tail -60 gpurun_out/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 2>/dev/null | tail -1 | cut -c1-200 || exit 1
