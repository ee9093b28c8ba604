#!/bin/bash
# round 5 final (fold tables, G2 segment rule): the whole GPU suite + smoke, the rocprofv3 trace and PMC
# passes of the default bench command, the default bench line
PYTEST_ARGS="--timeout 600 --timeout-method thread" GPU_TEST_TIMEOUT=1000 bash tools/gpu_check.sh || exit $?
bash tools/profile_round.sh r05ao || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_full_r05ao.log 2>&1
