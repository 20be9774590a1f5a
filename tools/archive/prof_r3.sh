#!/bin/bash
# round-3 rocprofv3 evidence: async groups concurrency, pipelined predict (kernels + copies), Otto fp32 step
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_async -o run -- python3 $R/bench.py --mode asynchronous --frequency epoch --steps 500 --warmup 50 > $R/gpurun_out/prof_async.txt 2>&1 || { echo async prof failed; tail $R/gpurun_out/prof_async.txt; exit 1; }
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/prof_predict -o run -- python3 $R/bench.py --task predict --steps 5 --warmup 1 > $R/gpurun_out/prof_predict.txt 2>&1 || { echo predict prof failed; exit 1; }
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_otto -o run -- python3 $R/bench.py --model otto --steps 200 --warmup 20 > $R/gpurun_out/prof_otto.txt 2>&1 || { echo otto prof failed; exit 1; }
cd $R
python tools/rocpd_overlap.py gpurun_out/prof_async/run_results.db persist | tail -4
python tools/rocpd_summary.py gpurun_out/prof_otto/run_results.db gpurun_out/otto_fp32_r3_kernel_stats.csv --top 8
tail -1 gpurun_out/prof_async.txt | cut -c1-150; tail -1 gpurun_out/prof_predict.txt | cut -c1-150; tail -1 gpurun_out/prof_otto.txt | cut -c1-150
