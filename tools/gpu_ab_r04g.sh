#!/bin/bash
# round 4: parity of the BLS12-381 G1 28-bit reductions, the reordered pair
# additions and the multi-device NTT on any device list; then the BLS12-381
# G1 / G2 reductions A/B in one process (set_variant bit 22 = FIPS reductions).
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_msm.py tests/test_gpu_groth16.py tests/test_gpu_ntt.py > gpurun_out/t_r04g.log 2>&1 &&
timeout -k 10 300 python tools/tune_msm.py --curve bls12_381_g1 --log-n 22 24 --variants 0 4194304 --rounds 2 \
  > gpurun_out/ab_bls_g1_reduce.log 2>&1 &&
timeout -k 10 300 python tools/tune_msm.py --curve bls12_381_g2 --log-n 22 --variants 0 4194304 --rounds 2 \
  > gpurun_out/ab_bls_g2_reduce2.log 2>&1 &&
timeout -k 10 300 python tools/tune_msm.py --curve bn254_g2 --log-n 20 --variants 0 4194304 --rounds 2 \
  > gpurun_out/ab_g2_reduce2.log 2>&1
