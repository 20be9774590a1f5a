#!/bin/bash
# 2-rank (one shared GPU) persistent-plan SparkModel sync test + bench rehearsal with
# persistent grids of half the CUs each (the lazy-image averaging on the multi-rank path)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_peer_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_peer.txt 2>&1 || { echo "tests failed: $?"; tail -60 gpurun_out/t_peer.txt; exit 1; }
grep -E "PASS|FAIL" gpurun_out/t_peer.txt | tail -20
ELEPHAS_AMD_PERSIST=1 ELEPHAS_AMD_PERSIST_CUS=128 ELEPHAS_AMD_DIST_BACKEND=gloo ELEPHAS_AMD_P2P_ANY_BACKEND=1 timeout -k 10 240 python bench.py --gpus 2 --workers-per-gpu 4 --steps 200 --warmup 20 > gpurun_out/rehearsal_persist2.txt 2>&1 || { tail -30 gpurun_out/rehearsal_persist2.txt; exit 1; }
tail -1 gpurun_out/rehearsal_persist2.txt | cut -c1-1500
