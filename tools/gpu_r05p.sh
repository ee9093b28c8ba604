#!/bin/bash
# round 5: the whole GPU suite + smoke after the recode / NTT changes, then the
# default bench line
PYTEST_ARGS="--timeout 600 --timeout-method thread" GPU_TEST_TIMEOUT=1000 bash tools/gpu_check.sh || exit $?
mkdir -p gpurun_out/r05p
timeout -k 10 400 python bench.py > gpurun_out/r05p/bench_full.log 2>&1
