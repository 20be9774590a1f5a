#!/bin/bash
# per-step sync exchange: skew vs post-arrival latency
mkdir -p gpurun_out
. tools/gpu_step.sh
step r5t_sync_stamps_ag 120 python tools/persist_stamps.py 8 64 8 -1 float32 sync
step r5t_sync_stamps_rs 120 env ELEPHAS_AMD_XCHG_RS=1 python tools/persist_stamps.py 8 64 8 -1 float32 sync
step r5t_v1_stamps 120 python tools/persist_stamps.py 8 64 8 0 float32
