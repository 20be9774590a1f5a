#!/bin/bash
# full GPU suite + smoke + rocprofv3 kernel trace of the headline bench (evidence for profiles/)
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4.txt 2>&1; rc=$?
tail -15 gpurun_out/gpu_tests_r4.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit 1; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o mnist_r4 -- python bench.py --gpus 1 --steps 300 --warmup 30 --no-sub > gpurun_out/prof_bench.txt 2>&1 || exit 1
tail -1 gpurun_out/prof_bench.txt | cut -c1-200
find gpurun_out/prof -name "*kernel_stats.csv" | head -3
