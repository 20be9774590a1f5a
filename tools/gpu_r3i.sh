#!/bin/bash
# persistent chunks as single launches (remainder included), 128-step chunks:
# persistent tests, driver-shape bench x3, 2000 steps, kernel trace of the driver shape
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_persist_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_persist.txt 2>&1 || { echo "tests failed: $?"; tail -40 gpurun_out/t_persist.txt; exit 1; }
tail -2 gpurun_out/t_persist.txt
O=gpurun_out/r3i.jsonl; : > $O
for i in 1 2 3; do timeout -k 10 120 python bench.py --steps 20 --warmup 5 --out $O > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }; done
timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --out $O > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
ELEPHAS_AMD_PERSIST_CHUNK=64 timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --out $O > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
python -c "
import json
for l in open('$O'): d=json.loads(l); print(d['steps'], d['ms_per_step'], round(d['value']))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_drv -o k -- python $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_drv.log 2>&1
echo prof rc=$?
