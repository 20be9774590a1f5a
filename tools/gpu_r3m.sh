#!/bin/bash
# kernel trace of async frequency='batch' (8 independent groups) and hogwild, 1 GPU
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_async -o k -- python $R/bench.py --mode asynchronous --frequency batch --steps 100 --warmup 20 > $R/gpurun_out/prof_async.log 2>&1
echo prof rc=$?
tail -1 $R/gpurun_out/prof_async.log | cut -c1-300
