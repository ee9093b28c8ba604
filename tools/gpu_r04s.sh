#!/bin/bash
# round 4: the batch window rule (c = 0) against c 5..11 at every length 2^10..2^16, then batch parity
mkdir -p gpurun_out
timeout -k 10 500 python tools/batch_probe.py --log-len 10 11 12 13 14 15 16 --count 8 32 128 --reps 3 \
  --c 0 5 6 7 8 9 10 11 > gpurun_out/batch_probe4.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  "tests/test_gpu_msm.py::test_msm_batch_vs_oracle" tests/test_gpu_kzg.py > gpurun_out/t_batch2.log 2>&1
