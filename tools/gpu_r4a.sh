#!/bin/bash
# round-4 baseline on a fresh box: bench driver shape, batch granularity, stamps of the persistent step
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r4a.log; : > $O
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 2>/dev/null | tail -n1 >> $O || exit 1
timeout -k 10 150 python bench.py --gpus 1 --steps 2000 --warmup 50 2>/dev/null | tail -n1 >> $O || exit 1
timeout -k 10 150 python bench.py --gpus 1 --steps 200 --warmup 20 --granularity batch 2>/dev/null | tail -n1 >> $O || exit 1
timeout -k 10 150 python tools/persist_stamps.py 8 64 8 > gpurun_out/stamps_r4a.txt 2>&1 || exit 1
cut -c1-160 $O
tail -3 gpurun_out/stamps_r4a.txt
