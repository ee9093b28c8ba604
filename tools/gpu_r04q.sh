#!/bin/bash
# round 4: the batched MSM with the per-MSM window size -- parity, then batched vs separate
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  "tests/test_gpu_msm.py::test_msm_batch_vs_oracle" tests/test_gpu_kzg.py > gpurun_out/t_batch.log 2>&1 &&
timeout -k 10 300 python tools/batch_probe.py --log-len 10 12 14 16 --count 8 32 > gpurun_out/batch_probe2.log 2>&1
