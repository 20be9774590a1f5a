#!/bin/bash
# Layer-0 split-K slab count of the row-chain plan (ELEPHAS_AMD_RC_SPLIT, 0 = auto = ceil(K/112))
set -u
O=gpurun_out/rc_split.log
for w in 8 1; do
  for s in 0 4 5 10 13; do
    echo "== workers $w RC_SPLIT=$s" >> $O
    ELEPHAS_AMD_RC_SPLIT=$s timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --workers-per-gpu $w >> $O 2>&1 || exit 1
  done
done
