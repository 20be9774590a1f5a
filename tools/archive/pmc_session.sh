#!/bin/bash
# PMC counters for the training step kernels (counters only, no tracing domains).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_IFETCH_LEVEL \
  --output-format csv -d "$OUT/pmcA" -o k -- python "$ROOT/bench.py" --steps 40 --warmup 8 > "$OUT/pmcA.log" 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS \
  --output-format csv -d "$OUT/pmcB" -o k -- python "$ROOT/bench.py" --steps 40 --warmup 8 > "$OUT/pmcB.log" 2>&1 || exit $?
