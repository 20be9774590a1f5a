#!/bin/bash
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $OUT/pmc_list.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAVES SQ_INSTS_VALU --output-format csv -d "$OUT/pmc1" -o k -- python "$ROOT/bench.py" --steps 50 --warmup 10 > $OUT/pmc1.log 2>&1
echo rc=$?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU --output-format csv -d "$OUT/pmc2" -o k -- python "$ROOT/bench.py" --steps 50 --warmup 10 > $OUT/pmc2.log 2>&1
echo rc=$?
