#!/bin/bash
# the whole GPU suite with kernels serialised (plan-expectation failures without timing races)
mkdir -p gpurun_out
. tools/gpu_step.sh
AMD_SERIALIZE_KERNEL=3 step r5m_tests_serial 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
