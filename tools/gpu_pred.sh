#!/bin/bash
# Wide / MNIST predict A/B: host fp32->bf16 packing vs fp32 DMA + device conversion
set -o pipefail
P=gpurun_out/pred_ab.log; : > $P
for arm in 0 1; do
  for m in "--model wide --policy mixed_bfloat16" "--model mnist"; do
    ELEPHAS_AMD_INFER_DEVICE_CVT=$arm timeout -k 10 200 python bench.py --task predict $m --steps 10 --warmup 2 2>/dev/null | tail -n1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('device_cvt=$arm $m', d['ms_per_step'], round(d['value']))" >> $P || exit 1
  done
done
cat $P
