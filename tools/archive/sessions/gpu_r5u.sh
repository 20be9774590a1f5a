#!/bin/bash
mkdir -p gpurun_out
. tools/gpu_step.sh
step r5u_big_ab 300 python tools/big_ab.py 4,7,5
