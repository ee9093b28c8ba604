#!/bin/bash
# GPU-box check script: smoke, then the gpu tests; stops at the first step that
# faulted/aborted/timed out (rc not in {0,1}).
mkdir -p gpurun_out
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 ${GPU_TEST_TIMEOUT:-600} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" | tee -a gpurun_out/gpu_tests.log
exit $rc
