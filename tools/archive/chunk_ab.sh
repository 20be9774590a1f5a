#!/bin/bash
# steps per captured hipGraph (ELEPHAS_AMD_GRAPH_CHUNK) A/B, MNIST fp32
set -u
O=gpurun_out/chunk_ab.log
for round in 1 2; do
  for c in 16 64; do
    echo "== round $round CHUNK=$c" >> $O
    ELEPHAS_AMD_GRAPH_CHUNK=$c timeout -k 10 120 python bench.py --steps 2000 --warmup 200 >> $O 2>&1 || exit 1
    ELEPHAS_AMD_GRAPH_CHUNK=$c timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 >> $O 2>&1 || exit 1
  done
done
