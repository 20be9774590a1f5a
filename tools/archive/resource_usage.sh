#!/bin/bash
# register / scratch / LDS use of the persistent kernel instances (compiler remarks)
# usage: tools/resource_usage.sh [source (default csrc/kernels/persist.hip)] [kernel-name filter]
SRC=${1:-csrc/kernels/persist.hip}
PAT=${2:-mlp_persist_kernel}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc --cuda-device-only -c "$SRC" -o /tmp/ru.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk -v pat="$PAT" '/Function Name:/ {keep = index($0, pat) > 0; if (keep) print ""} keep && /Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|LDS Size|SGPRs:/' |
  sed -E 's/^.*remark: //'
