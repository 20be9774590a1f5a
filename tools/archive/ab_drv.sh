#!/bin/bash
# A/B two native builds (tmp_so/old.so vs tmp_so/new.so) on the driver shape and 2000 steps, 3 rounds
SO=elephas_amd/_C.cpython-310-x86_64-linux-gnu.so
mkdir -p gpurun_out; : > gpurun_out/ab_drv.log
for round in 1 2 3; do for v in old new; do cp tmp_so/$v.so $SO
  for a in "--steps 20 --warmup 5" "--steps 2000 --warmup 200"; do
    timeout -k 10 200 python bench.py $a 2>/dev/null | tail -n1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$round $v $a', d['ms_per_step'])" >> gpurun_out/ab_drv.log || exit 1
  done
done; done
cp tmp_so/new.so $SO
cat gpurun_out/ab_drv.log
