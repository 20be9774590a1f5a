#!/bin/bash
# tools/big_ab.py plus a PMC pass (L2 hits, waits, MFMA busy)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
timeout -k 10 120 python "$ROOT/tools/big_ab.py" >> "$OUT/big_ab.log" 2>&1 || exit $?
if [ "${PMC:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum \
    --output-format csv -d "$OUT/bigpmc" -o k -- python "$ROOT/tools/big_ab.py" > "$OUT/bigpmc.log" 2>&1 || exit $?
fi
