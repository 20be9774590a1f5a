#!/bin/bash
# End-of-round-4 record: smoke, 1-GPU sweep, inference probe, kernel-trace stats of the
# headline, Otto and Wide, persistent-kernel stamps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
bash tools/sweep.sh || exit 1
timeout -k 10 300 python tools/infer_probe.py > gpurun_out/infer_probe_r4.txt 2>&1 || exit 1
grep -v -E "amdgpu.ids|Warning|from elephas" gpurun_out/infer_probe_r4.txt
timeout -k 10 150 python tools/persist_stamps.py 8 64 8 > gpurun_out/stamps_final_r4.txt 2>&1 || exit 1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pf_mnist -o k -- python $R/bench.py --steps 300 --warmup 30 --no-sub > $R/gpurun_out/pf_mnist.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pf_otto -o k -- python $R/bench.py --model otto --batch 128 --steps 300 --warmup 30 --no-sub > $R/gpurun_out/pf_otto.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pf_wide -o k -- python $R/bench.py --model wide --policy mixed_bfloat16 --workers-per-gpu 1 --batch 1024 --steps 40 --warmup 8 --no-sub > $R/gpurun_out/pf_wide.log 2>&1 || exit 1
echo prof ok
