set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --model wide --steps 30 --warmup 5 --workers-per-gpu 1 --batch 1024 > gpurun_out/bench_wide.log 2>&1 &&
timeout -k 10 300 python bench.py --model wide --steps 30 --warmup 5 --workers-per-gpu 1 --batch 1024 --granularity batch > gpurun_out/bench_wide_batch.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > gpurun_out/bench_default.log 2>&1
