#!/bin/bash
# persistent chunk = kernel + one post node (flag clear + counter advance): tests, A/B vs the
# memset + kernel + advance build on the driver shape, async batch numbers
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1 || { echo "tests failed: $?"; tail -60 gpurun_out/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/gpu_tests.txt
bash tools/ab_drv.sh || exit 1
O=gpurun_out/r3x.log; : > $O
run() { timeout -k 10 200 python bench.py "$@" 2>/dev/null | tail -n1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*', d['ms_per_step'], round(d['value']))" >> $O; }
for v in old new old new; do cp tmp_so/$v.so elephas_amd/_C.cpython-310-x86_64-linux-gnu.so
  echo "== $v" >> $O
  run --mode asynchronous --frequency batch --steps 300 --warmup 30 || exit 1
done
cp tmp_so/new.so elephas_amd/_C.cpython-310-x86_64-linux-gnu.so
cat $O
