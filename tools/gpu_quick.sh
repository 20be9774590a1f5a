set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_native_gpu.py -v -m gpu --timeout 120 --timeout-method thread -x -k "not nothing" > gpurun_out/t_rc.log 2>&1; rc=$?
tail -4 gpurun_out/t_rc.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python tools/stamps.py 8 mnist 64 float32 > gpurun_out/stamps_rc.txt 2>&1 || exit $?
grep -v Warning gpurun_out/stamps_rc.txt | grep -v nanmedian
timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > gpurun_out/b_f32.log 2>&1 || exit $?
tail -1 gpurun_out/b_f32.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_rc -o k -- python $GRAFT_REPO_ROOT/bench.py --steps 300 --warmup 30 > $GRAFT_REPO_ROOT/gpurun_out/prof_rc.log 2>&1
echo prof rc=$?
python $GRAFT_REPO_ROOT/tools/trace_steps.py $GRAFT_REPO_ROOT/gpurun_out/prof_rc/k_kernel_trace.csv 600 | head -5
