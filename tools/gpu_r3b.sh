#!/bin/bash
# round-3 probes: inference breakdown, stream overlap (persistent on / off), Otto fp32 stamps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/infer_probe.py > gpurun_out/infer_probe.txt 2>&1; echo "infer rc $?"; cat gpurun_out/infer_probe.txt | grep -v amdgpu.ids
timeout -k 10 180 python tools/stream_probe.py > gpurun_out/stream_probe.txt 2>&1 || { echo "stream probe failed $?"; tail gpurun_out/stream_probe.txt; exit 1; }
cat gpurun_out/stream_probe.txt | grep -v amdgpu.ids
ELEPHAS_AMD_PERSIST=0 timeout -k 10 180 python tools/stream_probe.py > gpurun_out/stream_probe_p0.txt 2>&1 || exit 1
cat gpurun_out/stream_probe_p0.txt | grep -v amdgpu.ids
PROBE_GRAPH=0 ELEPHAS_AMD_PERSIST=0 timeout -k 10 180 python tools/stream_probe.py 1 4 > gpurun_out/stream_probe_eager.txt 2>&1 || exit 1
cat gpurun_out/stream_probe_eager.txt | grep -v amdgpu.ids
timeout -k 10 120 python tools/stamps.py 8 otto 128 float32 > gpurun_out/stamps_otto_fp32.txt 2>&1; echo "stamps rc $?"
cd /tmp && export TMPDIR=/tmp
ELEPHAS_AMD_PERSIST=0 timeout -k 10 180 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof_streams -o run -- python3 $GRAFT_REPO_ROOT/tools/stream_probe.py 4 > $GRAFT_REPO_ROOT/gpurun_out/prof_streams.txt 2>&1 && echo streams prof ok
cd $GRAFT_REPO_ROOT && python tools/rocpd_overlap.py gpurun_out/prof_streams/run_results.db
