#!/bin/bash
# bench rehearsal of the multi-GPU path with persistent grids (2 ranks sharing the GPU, half
# the CUs each, 4 workers per rank) + the default 1-GPU bench line
set -o pipefail
mkdir -p gpurun_out
ELEPHAS_AMD_PERSIST=1 ELEPHAS_AMD_PERSIST_CUS=128 ELEPHAS_AMD_DIST_BACKEND=gloo ELEPHAS_AMD_P2P_ANY_BACKEND=1 timeout -k 10 240 python bench.py --gpus 2 --workers-per-gpu 4 --steps 200 --warmup 20 > gpurun_out/rehearsal_persist2.txt 2>&1 || { tail -30 gpurun_out/rehearsal_persist2.txt; exit 1; }
tail -1 gpurun_out/rehearsal_persist2.txt
timeout -k 10 120 python bench.py > gpurun_out/bench_default.txt 2>&1 || { tail -30 gpurun_out/bench_default.txt; exit 1; }
tail -1 gpurun_out/bench_default.txt
