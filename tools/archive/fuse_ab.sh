#!/bin/bash
# Fused layer-0 slabs + row chain (ELEPHAS_AMD_RC_FUSE=1): GPU tests with it on, then A/B
set -u
O=gpurun_out
ELEPHAS_AMD_RC_FUSE=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t_fuse.log 2>&1 || exit 1
for round in 1 2; do
  for v in 0 1; do
    for w in 8 1; do
      echo "== round $round RC_FUSE=$v workers $w" >> $O/fuse_ab.log
      ELEPHAS_AMD_RC_FUSE=$v timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --workers-per-gpu $w >> $O/fuse_ab.log 2>&1 || exit 1
    done
  done
done
ELEPHAS_AMD_RC_FUSE=1 timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 >> $O/fuse_ab.log 2>&1 || exit 1
