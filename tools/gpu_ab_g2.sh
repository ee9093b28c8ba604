#!/bin/bash
# GPU box: field/point/MSM/Groth16 parity of the current library, then an A/B
# against LIB_A on the G2 MSMs (BN254 G2 2^20/2^22, BLS12-381 G2 2^21).
export LIB_B=tachyon_amd/libtachyon_mi355x.so
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_field_ec.py tests/test_gpu_msm.py tests/test_gpu_groth16.py > gpurun_out/t_field_msm.log 2>&1 &&
bash tools/ab_libs.sh 2 --curve bn254_g2 --log-n 20 22 &&
bash tools/ab_libs.sh 1 --curve bls12_381_g2 --log-n 21
