#!/bin/bash
# round 4 (final library): the batched-MSM parity cases, then the default bench line
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  "tests/test_gpu_msm.py::test_msm_batch_vs_oracle" > gpurun_out/t_batch4.log 2>&1 &&
timeout -k 10 900 python -u bench.py > gpurun_out/bench_final.log 2>&1
