#!/bin/bash
# round 5: library communicators (RCCL world 1, host-staged world 2) + the dist tests
mkdir -p gpurun_out/r05b
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_comm.py tests/test_gpu_dist.py > gpurun_out/r05b/tests.log 2>&1
