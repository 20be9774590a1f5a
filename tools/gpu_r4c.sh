#!/bin/bash
# follow-up: stamps of V2 / V1, the fixed sync test, bf16 diagnostics
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python tools/persist_stamps.py 8 64 8 1 > gpurun_out/stamps_v2_r4c.txt 2>&1 || exit 1
timeout -k 10 150 python tools/persist_stamps.py 8 64 8 0 > gpurun_out/stamps_v1_r4c.txt 2>&1 || exit 1
grep -v "amdgpu.ids\|RuntimeWarning\|from elephas" gpurun_out/stamps_v2_r4c.txt | tail -26
grep "period" gpurun_out/stamps_v1_r4c.txt
timeout -k 10 300 python -u -m pytest tests/test_persist_gpu.py -v --timeout 120 --timeout-method thread -k "sync or bf16" > gpurun_out/t_sync.txt 2>&1; rc=$?
grep -E "PASSED|FAILED|^E   " gpurun_out/t_sync.txt | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
timeout -k 10 200 python tools/bf16_check.py 0.2 2>&1 | grep dropout
timeout -k 10 200 python tools/bf16_check.py 0 2>&1 | grep dropout
