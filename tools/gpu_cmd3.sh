set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_native_gpu.py -q --timeout 120 --timeout-method thread -k "deferred or deterministic or fused_tail" > gpurun_out/gpu_t3.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
ELEPHAS_AMD_FUSED=2 timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > gpurun_out/bench_f2.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > gpurun_out/bench_f0.log 2>&1
