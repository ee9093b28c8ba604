#!/bin/bash
# round 4: batched MSM under a forced window size, and the multi-device NTT domain again
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  "tests/test_gpu_msm.py::test_msm_batch_forced_window_bits" "tests/test_gpu_msm.py::test_msm_batch_vs_oracle" \
  "tests/test_gpu_ntt.py::test_multi_device_domain_logical" "tests/test_gpu_ntt.py::test_multi_device_domain_refused" \
  > gpurun_out/t_r04x.log 2>&1
