#!/bin/bash
# End-of-round-3 record: smoke, 1-GPU sweep, kernel-trace stats of the headline, Otto and Wide
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
bash tools/sweep.sh || exit 1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pf_mnist -o k -- python $R/bench.py --steps 300 --warmup 30 > $R/gpurun_out/pf_mnist.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pf_otto -o k -- python $R/bench.py --model otto --batch 128 --steps 300 --warmup 30 > $R/gpurun_out/pf_otto.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pf_wide -o k -- python $R/bench.py --model wide --policy mixed_bfloat16 --workers-per-gpu 1 --batch 1024 --steps 40 --warmup 8 > $R/gpurun_out/pf_wide.log 2>&1 || exit 1
echo prof ok
