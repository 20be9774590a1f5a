#!/bin/bash
# persistent V2 iteration: persist GPU tests, headline bench (A/B by env), stamps
# usage: tools/gpu_r4f.sh [ENV=VAL ...]   (each ENV=VAL adds a B arm to the bench A/B)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_persist_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/t_persist.txt 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/t_persist.txt | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit 1; fi
O=gpurun_out/r4f.log; : > $O
run() { timeout -k 10 150 python bench.py --no-sub "$@" 2>/dev/null | tail -n1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$*', d['ms_per_step'], round(d['value']), (c.get('engine') or '')[:90])" >> $O; }
run --gpus 1 --steps 20 --warmup 5 || exit 1
run --gpus 1 --steps 2000 --warmup 50 || exit 1
for kv in "$@"; do
  env "$kv" true || exit 1
  echo "arm $kv" >> $O
  export "$kv"
  run --gpus 1 --steps 20 --warmup 5 || exit 1
  run --gpus 1 --steps 2000 --warmup 50 || exit 1
  unset "${kv%%=*}"
done
cat $O
timeout -k 10 150 python tools/persist_stamps.py 8 64 8 > gpurun_out/stamps_r4f.txt 2>&1 || exit 1
grep -v -E "amdgpu.ids|Warning|from elephas" gpurun_out/stamps_r4f.txt | tail -32
[ -n "$PRED" ] && { bash tools/gpu_pred.sh || exit 1; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_drv4 -o k -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-sub > gpurun_out/prof_drv4.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/prof_drv4/**/k_kernel_trace.csv', recursive=True) + glob.glob('gpurun_out/prof_drv4/k_kernel_trace.csv')
rows = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r['Start_Timestamp']))
t0 = int(rows[-10]['Start_Timestamp'])
for r in rows[-10:]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print(f"{(s - t0) / 1000:9.1f} {(e - s) / 1000:8.1f}  {r['Kernel_Name'][:80]}")
PY
