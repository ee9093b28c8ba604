#!/bin/bash
# round 4: the new accumulation-chunk rule (K x2 for 2^22 < entries <= 2^25) across
# sizes and groups; MSM parity; onesweep tile shapes (bits 4-5) and recode scalars
# per thread (bits 8-9) at 2^24 / 2^26
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_msm.py \
  tests/test_gpu_groth16.py > gpurun_out/t_krule.log 2>&1 &&
timeout -k 10 300 python tools/tune_msm.py --curve bn254_g1 --log-n 16 17 18 19 20 21 22 --rounds 2 > gpurun_out/krule_g1.log 2>&1 &&
timeout -k 10 300 python tools/tune_msm.py --curve bn254_g2 --log-n 20 21 --rounds 2 > gpurun_out/krule_g2.log 2>&1 &&
timeout -k 10 300 python tools/tune_msm.py --curve bls12_381_g1 --log-n 20 21 --rounds 2 > gpurun_out/krule_bls.log 2>&1 &&
timeout -k 10 500 python tools/tune_msm.py --curve bn254_g1 --log-n 24 26 --variants 0 16 32 48 256 512 768 8388608 --rounds 2 \
  > gpurun_out/tune_sort_recode.log 2>&1
