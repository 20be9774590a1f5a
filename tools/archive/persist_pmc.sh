#!/bin/bash
# PMC passes over the persistent-plan bench (one counter group per pass).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
grep -iE "SQC|ICACHE|IFETCH" "$OUT/counters.txt" | head -40 > "$OUT/counters_sqc.txt" || true
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/pmc_$name" -o p -- \
    python3 "$ROOT/bench.py" --steps 200 --warmup 20 > "$OUT/pmc_$name.log" 2>&1
  echo "$name rc=$?"
}
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU
pass ic SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE
