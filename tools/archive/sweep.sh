#!/bin/bash
# 1-GPU bench sweep: one JSON line per config into gpurun_out/sweep.jsonl
set -o pipefail
O=gpurun_out/sweep.jsonl
mkdir -p gpurun_out; : > $O
run() { echo "== $*" >&2; timeout -k 10 240 python bench.py "$@" --out $O > gpurun_out/sweep_last.log 2>&1 || { echo "FAILED: $*"; tail -20 gpurun_out/sweep_last.log; exit 1; }; }
run --steps 20 --warmup 5
run --steps 2000 --warmup 200
run --workers-per-gpu 1 --steps 2000 --warmup 200
run --granularity batch --steps 500 --warmup 50
run --policy mixed_bfloat16 --steps 500 --warmup 50
run --task fit --steps 5 --warmup 2
run --mode asynchronous --frequency epoch --steps 500 --warmup 50
run --mode asynchronous --frequency batch --steps 300 --warmup 30
run --task predict --steps 10 --warmup 2
run --model otto --workers-per-gpu 8 --batch 128 --steps 200 --warmup 20
run --task fit --model otto --steps 3 --warmup 1
run --task predict --model wide --policy mixed_bfloat16 --steps 10 --warmup 2
run --model wide --policy mixed_bfloat16 --workers-per-gpu 1 --batch 1024 --steps 32 --warmup 8
echo sweep ok
