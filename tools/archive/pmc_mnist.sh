#!/bin/bash
# PMC pass over the fp32 MNIST step (headline config): where the waves' cycles go
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS \
  --output-format csv -d "$OUT/mpmc" -o m -- python "$ROOT/bench.py" --steps 200 --warmup 20 > "$OUT/mpmc.log" 2>&1
