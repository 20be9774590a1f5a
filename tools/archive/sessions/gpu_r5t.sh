#!/bin/bash
mkdir -p gpurun_out
. tools/gpu_step.sh
step r5t_big_variants 300 python tools/big_variants.py
step r5t_big_variants2 300 python tools/big_variants.py
