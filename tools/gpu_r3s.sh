#!/bin/bash
# PS pull-into-replicas test + PMC passes over the persistent MNIST kernel (the headline)
set -o pipefail
mkdir -p gpurun_out
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 300 python -u -m pytest tests/test_native_gpu.py -x -q --timeout 120 --timeout-method thread -k "ps_" > gpurun_out/t_ps.txt 2>&1 || { echo "tests failed: $?"; tail -40 gpurun_out/t_ps.txt; exit 1; }
tail -1 gpurun_out/t_ps.txt
cd /tmp && export TMPDIR=/tmp
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$R/gpurun_out/pmcp_$name" -o p -- \
    python3 "$R/bench.py" --steps 300 --warmup 30 > "$R/gpurun_out/pmcp_$name.log" 2>&1
  echo "$name rc=$?"
}
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS || exit 1
pass mem SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum || exit 1
python3 $R/tools/pmc_summary.py $(find $R/gpurun_out/pmcp_sq $R/gpurun_out/pmcp_mem -name "*counter_collection.csv") > $R/gpurun_out/pmc_persist_r3.txt
grep -A20 persist $R/gpurun_out/pmc_persist_r3.txt | head -24
