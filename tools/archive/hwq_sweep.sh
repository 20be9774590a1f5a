#!/bin/bash
# async / multi-group throughput vs the number of HIP hardware queues per process
set -u
O=gpurun_out/hwq_sweep.log
for q in 8 16; do
  for args in "--mode asynchronous --frequency epoch" "--mode asynchronous --frequency epoch --async-groups 4" "--mode asynchronous --frequency batch"; do
    echo "== GPU_MAX_HW_QUEUES=$q $args" >> $O
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --steps 1000 --warmup 100 $args >> $O 2>&1 || exit 1
  done
done
