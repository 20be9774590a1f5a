#!/bin/bash
# 16 hardware queues by default: full sweep + async batch-frequency row-chain vs persistent
set -o pipefail
mkdir -p gpurun_out
bash tools/sweep.sh || exit 1
O=gpurun_out/sweep5.jsonl; : > $O
ELEPHAS_AMD_PERSIST=0 timeout -k 10 240 python bench.py --mode asynchronous --frequency batch --steps 300 --warmup 30 --out $O > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
tail -1 $O | cut -c1-160
timeout -k 10 240 python bench.py --mode hogwild --frequency batch --steps 300 --warmup 30 --out $O > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
tail -1 $O | cut -c1-160
