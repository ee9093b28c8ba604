#!/bin/bash
# GPU box: the whole GPU suite + smoke, then the rocprofv3 evidence of one
# round (tools/profile_round.sh) and the default bench line.
#   bash tools/gpu_round_evidence.sh <tag>
TAG=${1:?tag}
GPU_TEST_TIMEOUT=700 bash tools/gpu_check.sh &&
bash tools/profile_round.sh $TAG &&
timeout -k 10 400 python bench.py > gpurun_out/bench_full_$TAG.log 2>&1
