#!/bin/bash
# One GPU session: tests, smoke, benchmarks, kernel profile.  Stops at the first
# fault/timeout (exit codes >1 other than test failures).
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a "$OUT/session.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/session.log"
  tail -3 "$OUT/$name.log" | tee -a "$OUT/session.log"
  return $rc
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step gpu_tests 900 python -u -m pytest tests -v -m gpu -x --timeout 120 --timeout-method thread; rc=$?
  [ $rc -gt 1 ] && exit $rc
  step smoke 180 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
  step bench_default 300 python bench.py --steps 2000 --warmup 200 || exit $?
  step bench_w1 300 python bench.py --steps 2000 --warmup 200 --workers-per-gpu 1 || exit $?
  step bench_batch 300 python bench.py --steps 1000 --warmup 100 --granularity batch || exit $?
  step bench_bf16 300 python bench.py --steps 1000 --warmup 100 --policy mixed_bfloat16 || exit $?
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
  cd /tmp && export TMPDIR=/tmp
  echo "== rocprof" | tee -a "$OUT/session.log"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- \
      python "$ROOT/bench.py" --steps 300 --warmup 30 > "$OUT/rocprof.log" 2>&1
  echo "   rc=$?" | tee -a "$OUT/session.log"
fi
