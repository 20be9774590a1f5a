#!/bin/bash
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
cd "$ROOT"
timeout -k 10 120 python bench.py --steps 1000 --warmup 100 > $OUT/ka_default.log 2>&1 || exit 1
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 120 python bench.py --steps 1000 --warmup 100 > $OUT/ka_dev.log 2>&1 || exit 1
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 120 python bench.py --steps 1000 --warmup 100 > $OUT/ka_host.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_ka" -o k -- python "$ROOT/bench.py" --steps 200 --warmup 20 > $OUT/prof_ka.log 2>&1
grep -h value $OUT/ka_*.log | cut -c1-200
