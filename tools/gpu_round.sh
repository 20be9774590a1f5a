#!/bin/bash
# one GPU session: full GPU test suite, 1-GPU bench, 2-rank same-GPU rehearsal, kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1 || { echo "tests failed: $?"; tail -30 gpurun_out/gpu_tests.txt; exit 1; }
tail -3 gpurun_out/gpu_tests.txt
timeout -k 10 120 python bench.py > gpurun_out/bench1.txt 2>&1 && tail -1 gpurun_out/bench1.txt
ELEPHAS_AMD_DIST_BACKEND=gloo ELEPHAS_AMD_P2P_ANY_BACKEND=1 timeout -k 10 300 python bench.py --gpus 2 --steps 200 --warmup 20 > gpurun_out/bench2r.txt 2>&1 && tail -1 gpurun_out/bench2r.txt
cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 512 --warmup 64 > $GRAFT_REPO_ROOT/gpurun_out/prof.txt 2>&1 && echo prof ok
