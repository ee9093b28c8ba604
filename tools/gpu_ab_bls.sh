#!/bin/bash
# GPU box: BLS12-381 field/point/MSM parity of the current library, then an
# A/B against LIB_A on the BLS12-381 G1 MSM (2^22 and 2^24).
export LIB_B=tachyon_amd/libtachyon_mi355x.so
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_field_ec.py tests/test_gpu_msm.py > gpurun_out/t_field_msm.log 2>&1 &&
bash tools/ab_libs.sh 2 --curve bls12_381_g1 --log-n 22 24
