#!/bin/bash
# round 4: MSM / Groth16 parity of the current library (BN254 G1 back to the
# reduced run start; the G2 reductions over the limb-field pairs), the G2
# reductions A/B in one process (set_variant bit 22 = the FIPS pair), then
# BN254 G1 and Groth16 against LIB_A, and the BN254 G2 window sizes 16-18.
export LIB_A=${LIB_A:-tachyon_amd/ab/lib_a.so} LIB_B=${LIB_B:-tachyon_amd/libtachyon_mi355x.so}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_msm.py tests/test_gpu_groth16.py > gpurun_out/t_r04f.log 2>&1 &&
timeout -k 10 300 python tools/tune_msm.py --curve bn254_g2 --log-n 20 22 --variants 0 4194304 --rounds 2 \
  > gpurun_out/ab_g2_reduce.log 2>&1 &&
timeout -k 10 300 python tools/tune_msm.py --curve bls12_381_g2 --log-n 22 --variants 0 4194304 --rounds 2 \
  > gpurun_out/ab_bls_g2_reduce.log 2>&1 &&
bash tools/ab_libs.sh 2 --curve bn254_g1 --log-n 24 26 &&
bash tools/gpu_ab_groth16.sh 3 &&
timeout -k 10 200 python tools/tune_msm.py --curve bn254_g2 --log-n 20 --c 16 17 18 > gpurun_out/tune_g2_2_20b.log 2>&1
