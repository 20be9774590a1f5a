#!/bin/bash
# GPU suite, probes (inference, stream concurrency), 1-GPU sweep, Otto fp32 stamps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1 || { echo "tests failed: $?"; tail -40 gpurun_out/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/gpu_tests.txt
timeout -k 10 120 python tools/infer_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/infer_probe.txt || exit 1
timeout -k 10 120 python tools/stream_micro.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/stream_micro.txt || exit 1
timeout -k 10 240 python tools/stream_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/stream_probe.txt || exit 1
ELEPHAS_AMD_PERSIST=0 timeout -k 10 240 python tools/stream_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/stream_probe_p0.txt || exit 1
timeout -k 10 120 python tools/stamps.py 8 otto 128 float32 2>&1 | grep "^launch" | tee gpurun_out/stamps_otto_fp32.txt || exit 1
bash tools/sweep.sh || exit 1
