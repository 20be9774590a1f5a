set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_native_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "deterministic or fused_tail or plain_gemm" > gpurun_out/gpu_tests3.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python tools/gemm_check.py > gpurun_out/gemm_check.log 2>&1
