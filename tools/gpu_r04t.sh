#!/bin/bash
# round 4: the final batch window rule -- batch parity, then batched vs separate at c = the rule
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  "tests/test_gpu_msm.py::test_msm_batch_vs_oracle" tests/test_gpu_kzg.py > gpurun_out/t_batch3.log 2>&1 &&
timeout -k 10 400 python tools/batch_probe.py --log-len 10 11 12 13 14 15 16 --count 8 32 128 --reps 5 \
  > gpurun_out/batch_probe5.log 2>&1
