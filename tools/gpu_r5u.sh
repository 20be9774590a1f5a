#!/bin/bash
# Wide 8 workers: per-launch in-kernel phase stamps of one step
mkdir -p gpurun_out
. tools/gpu_step.sh
step r5u_wide_stamps 240 python tools/stamps.py 8 wide 1024 mixed_bfloat16
