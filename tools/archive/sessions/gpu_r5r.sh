#!/bin/bash
# per-step sync (V1 roles) phase stamps; 256x256 schedule variants with the fixed epilogue
mkdir -p gpurun_out
. tools/gpu_step.sh
step r5r_sync_stamps 120 python tools/persist_stamps.py 8 64 8 -1 float32 sync
step r5r_v1_stamps 120 python tools/persist_stamps.py 8 64 8 0 float32
step r5r_big_variants 300 python tools/big_variants.py
