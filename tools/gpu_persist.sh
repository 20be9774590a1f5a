#!/bin/bash
# Persistent-plan session: its GPU tests, then the driver-shape bench with and without
# it (A/B in one box), then longer runs.  Stops at the first fault / timeout.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a "$OUT/session.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/session.log"
  tail -4 "$OUT/$name.log" | tee -a "$OUT/session.log"
  return $rc
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step persist_tests 400 python -u -m pytest tests/test_persist_gpu.py -v -x --timeout 120 --timeout-method thread
  rc=$?; [ $rc -gt 1 ] && exit $rc
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench_persist 180 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
  step bench_rowchain 180 env ELEPHAS_AMD_PERSIST=0 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
  step bench_persist_2000 180 python bench.py --steps 2000 --warmup 200 || exit $?
  step bench_persist_w1 180 python bench.py --steps 2000 --warmup 200 --workers-per-gpu 1 || exit $?
fi
