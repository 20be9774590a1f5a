#!/bin/bash
# Wide 8 workers: per-launch in-kernel phase stamps of one step
mkdir -p gpurun_out
. tools/gpu_step.sh
step r5u_wide_stamps 240 python tools/stamps.py 8 wide 1024 mixed_bfloat16
step r5u_host_overhead 120 python tools/host_overhead.py 20 30
