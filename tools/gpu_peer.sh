#!/bin/bash
# GPU session for the peer-memory paths: sharded PS + peer all-reduce tests (two
# processes sharing the GPU), the all-reduce microbenchmark (+ kernel trace of
# rank 0), async/hogwild benches.  MODE=tests|bench|all (default all).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a "$OUT/peer_session.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/peer_session.log"
  tail -4 "$OUT/$name.log" | cut -c1-600 | tee -a "$OUT/peer_session.log"
  return $rc
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step peer_ps_single 300 python -u -m pytest tests/test_native_gpu.py -v -x --timeout 120 --timeout-method thread -k "ps_" || exit $?
  step peer_tests 600 python -u -m pytest tests/test_peer_gpu.py -v -x --timeout 200 --timeout-method thread || exit $?
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step peer_bench 300 env ELEPHAS_AMD_PEER_PROF_DIR=$OUT/prof_peer python -c "import sys, json; sys.path.insert(0, 'tests'); from test_peer_gpu import _run; print(json.dumps(_run('bench')))" || exit $?
  for g in 8 2 1; do
    step async_bench_g$g 300 python bench.py --mode asynchronous --steps 320 --warmup 32 --async-groups $g || exit $?
  done
  step hogwild_bench 300 python bench.py --mode hogwild --steps 320 --warmup 32 || exit $?
  step async_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_async -o async -- python bench.py --mode asynchronous --steps 160 --warmup 16 || exit $?
fi
