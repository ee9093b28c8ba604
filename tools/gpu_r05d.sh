#!/bin/bash
# round 5 evidence: the whole GPU suite + smoke, the rocprofv3 trace and PMC
# passes of the default bench command (tools/profile_round.sh), the default
# bench line
PYTEST_ARGS="--timeout 600 --timeout-method thread" GPU_TEST_TIMEOUT=1000 bash tools/gpu_check.sh || exit $?
