#!/bin/bash
# Do several executors on several HIP streams of one process overlap?  Async epoch
# frequency with G groups, hipGraph dispatch settings vs eager launches.
set -u
O=gpurun_out/graph_dispatch.log
run() { echo "== $*" >> $O; timeout -k 10 200 "$@" >> $O 2>&1 || exit 1; }
B="python bench.py --steps 1000 --warmup 100 --mode asynchronous --frequency epoch"
run env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 $B --async-groups 2
run env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 $B --async-groups 4
run env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 $B
run $B --async-groups 4 --no-graph
run $B --async-groups 1 --no-graph
