#!/bin/bash
# A/B: layer-0 row-major weight image skipped in the row-chain DW launch (ELEPHAS_AMD_RC_LEAN)
set -u
O=gpurun_out/lean_ab.log
for round in 1 2; do
  for v in 0 1; do
    for w in 8 1; do
      echo "== round $round RC_LEAN=$v workers $w" >> $O
      ELEPHAS_AMD_RC_LEAN=$v timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --workers-per-gpu $w >> $O 2>&1 || exit 1
    done
  done
done
