#!/bin/bash
# Stamps of the fp32 MNIST step (1 and 8 workers) + the multi-rank rehearsal on one GPU
# (gloo control plane + IPC peer all-reduce, 2 processes sharing the GPU).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out
mkdir -p $O
timeout -k 10 120 python tools/stamps.py 1 mnist 64 float32 > $O/stamps_w1.txt 2>&1 || exit 1
timeout -k 10 120 python tools/stamps.py 8 mnist 64 float32 > $O/stamps_w8.txt 2>&1 || exit 1
ELEPHAS_AMD_DIST_BACKEND=gloo ELEPHAS_AMD_P2P_ANY_BACKEND=1 timeout -k 10 240 python bench.py --gpus 2 --steps 200 --warmup 20 > $O/rehearsal_fit.txt 2>&1 || exit 1
ELEPHAS_AMD_DIST_BACKEND=gloo ELEPHAS_AMD_P2P_ANY_BACKEND=1 timeout -k 10 240 python bench.py --gpus 2 --steps 200 --warmup 20 --granularity batch --workers-per-gpu 1 > $O/rehearsal_batch.txt 2>&1 || exit 1
