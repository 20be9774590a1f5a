#!/bin/bash
# Otto fp32 (8 x 128) step: default plan vs forced tile configs (merged DW+DX launches),
# plus per-launch stamps of each; results in gpurun_out/otto_ab.log
set -o pipefail
mkdir -p gpurun_out; O=gpurun_out/otto_ab.log; : > $O
for round in 1 2; do for v in -1 0 3 2; do
  ELEPHAS_AMD_GEMM_CFG=$v timeout -k 10 200 python bench.py --model otto --batch 128 --steps 1000 --warmup 100 2>/dev/null | tail -n1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$round CFG=$v otto', d['ms_per_step'], d['config'].get('launches_per_step'))" >> $O || exit 1
done; done
for v in 0 3; do
  echo "== stamps CFG=$v" >> $O
  ELEPHAS_AMD_GEMM_CFG=$v timeout -k 10 120 python tools/stamps.py 8 otto 128 float32 2>&1 | grep "^launch" >> $O || exit 1
done
cat $O
