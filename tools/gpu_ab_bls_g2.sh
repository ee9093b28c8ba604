#!/bin/bash
# GPU box: A/B of the BLS12-381 G2 MSM (2^21, 2^22) between the in-tree
# library (A) and LIB_B, after the G2 MSM parity tests of LIB_B.
export LIB_A=tachyon_amd/libtachyon_mi355x.so
mkdir -p gpurun_out
TACHYON_MI355X_LIB=$LIB_B timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_msm.py tests/test_gpu_field_ec.py -k "g2 or bls" > gpurun_out/t_libB.log 2>&1 &&
bash tools/ab_libs.sh 2 --curve bls12_381_g2 --log-n 21 22
