#!/bin/bash
# PMC passes over the THR GEMM (tools/gemm_pmc.py): MFMA busy, LDS conflicts, waits.
# One counter group per run (rocprofv3 does not split passes), counters only.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES \
  --output-format csv -d "$OUT/gpmcA" -o k -- python "$ROOT/tools/gemm_pmc.py" > "$OUT/gpmcA.log" 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS \
  --output-format csv -d "$OUT/gpmcB" -o k -- python "$ROOT/tools/gemm_pmc.py" > "$OUT/gpmcB.log" 2>&1 || exit $?
