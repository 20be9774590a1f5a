#!/bin/bash
# in-launch rank exchange: the 2-process tests, the persist GPU tests, and the per-step
# sync bench rehearsal on two ranks sharing the GPU
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_peer_gpu.py -v --timeout 200 --timeout-method thread -k "sync_inlaunch or spark_sync" > gpurun_out/t_xr.txt 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|assert|Error" gpurun_out/t_xr.txt | tail -20
[ $rc -ne 0 ] && { tail -60 gpurun_out/t_xr.txt; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_persist_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/t_persist.txt 2>&1; rc=$?
tail -2 gpurun_out/t_persist.txt
[ $rc -ne 0 ] && exit 1
for w in 2 8; do
  ELEPHAS_AMD_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 200 --warmup 20 --granularity batch --workers-per-gpu $w --no-sub > gpurun_out/xr_bench_w$w.txt 2>&1 || { tail -30 gpurun_out/xr_bench_w$w.txt; exit 1; }
  grep metric gpurun_out/xr_bench_w$w.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('W=$w', d['ms_per_step'], d['value'], c.get('sync'), '|', c.get('allreduce'), '| equal', c.get('theta_equal_on_all_ranks'), '|', c.get('engine')[:60])"
done
