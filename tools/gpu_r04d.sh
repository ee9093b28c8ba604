#!/bin/bash
# round 4: the whole GPU suite + smoke, then the default bench line
mkdir -p gpurun_out
PYTEST_ARGS="--timeout 300 --timeout-method thread" GPU_TEST_TIMEOUT=800 bash tools/gpu_check.sh || exit $?
timeout -k 10 420 python bench.py > gpurun_out/bench_r04d.log 2>&1
