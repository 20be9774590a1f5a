#!/bin/bash
# round-3 session: GPU suite, 1-GPU bench sweep, kernel traces of the MNIST (persistent) and Otto fp32 steps
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_round.sh || exit 1
bash tools/sweep.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_otto -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model otto --batch 128 --steps 200 --warmup 20 > $GRAFT_REPO_ROOT/gpurun_out/prof_otto.txt 2>&1 && echo otto prof ok
