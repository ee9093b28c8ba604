#!/bin/bash
# round 4: the G2 limb-pair window segments at one wave per SIMD (set_variant bit 23), A/B in one process
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  "tests/test_gpu_msm.py::test_msm_schedule_variants_agree" "tests/test_gpu_msm.py::test_msm_golden_g2_lane_pair" \
  > gpurun_out/t_wseg.log 2>&1 &&
timeout -k 10 400 python tools/tune_msm.py --curve bls12_381_g2 --log-n 22 24 --variants 0 8388608 --rounds 2 > gpurun_out/ab_wseg_bls_g2.log 2>&1 &&
timeout -k 10 300 python tools/tune_msm.py --curve bn254_g2 --log-n 20 22 --variants 0 8388608 --rounds 2 > gpurun_out/ab_wseg_bn_g2.log 2>&1
