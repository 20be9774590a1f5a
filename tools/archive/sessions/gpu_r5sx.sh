#!/bin/bash
# per-step sync exchange: all-gather + sum (batched loads) vs reduce-scatter + all-gather
mkdir -p gpurun_out
. tools/gpu_step.sh
step r5s_sync_stamps_ag 120 python tools/persist_stamps.py 8 64 8 -1 float32 sync
step r5s_sync_stamps_rs 120 env ELEPHAS_AMD_XCHG_RS=1 python tools/persist_stamps.py 8 64 8 -1 float32 sync
step r5s_sync_tests_ag 300 python -u -m pytest tests/test_persist_gpu.py tests/test_native_gpu.py -x -q -k sync --timeout 120 --timeout-method thread
step r5s_sync_tests_rs 300 env ELEPHAS_AMD_XCHG_RS=1 python -u -m pytest tests/test_persist_gpu.py tests/test_native_gpu.py -x -q -k sync --timeout 120 --timeout-method thread
step r5s_bench_ag 120 python bench.py --steps 20 --warmup 5
step r5s_bench_rs 120 env ELEPHAS_AMD_XCHG_RS=1 python bench.py --steps 20 --warmup 5
# Wide, 8 workers: tile order of the multi-replica 256x256 launches (interleaved)
step r5s_wide_g0a 150 python bench.py --model wide --policy mixed_bfloat16 --steps 20 --warmup 5 --no-sub
step r5s_wide_g1a 150 env ELEPHAS_AMD_BIG_GROUP=1 python bench.py --model wide --policy mixed_bfloat16 --steps 20 --warmup 5 --no-sub
step r5s_wide_g0b 150 python bench.py --model wide --policy mixed_bfloat16 --steps 20 --warmup 5 --no-sub
step r5s_wide_g1b 150 env ELEPHAS_AMD_BIG_GROUP=1 python bench.py --model wide --policy mixed_bfloat16 --steps 20 --warmup 5 --no-sub
