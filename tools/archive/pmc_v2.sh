#!/bin/bash
# PMC passes over the V2 persistent headline bench: SQ issue / wait mix and the
# instruction cache (one counter group per pass)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/pmcv2_$name" -o p -- \
    python3 "$ROOT/bench.py" --steps 300 --warmup 30 --no-sub > "$OUT/pmcv2_$name.log" 2>&1
  echo "$name rc=$?"
}
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA
pass ic SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE
python3 "$ROOT/tools/pmc_summary.py" $(find "$OUT/pmcv2_sq" "$OUT/pmcv2_ic" -name "*counter_collection.csv") 2>&1 | grep -A12 "mlp_persist" | head -40
