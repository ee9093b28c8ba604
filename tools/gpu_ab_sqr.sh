#!/bin/bash
# GPU box: field/point/MSM parity of the current library, then an A/B of it
# (LIB_B) against an earlier build (LIB_A, default ab/libA.so) on the MSM of
# every group, then the whole GPU suite.  Stops at the first failing step.
export LIB_A=${LIB_A:-ab/libA.so} LIB_B=tachyon_amd/libtachyon_mi355x.so
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_field_ec.py tests/test_gpu_msm.py > gpurun_out/t_field_msm.log 2>&1 &&
bash tools/ab_libs.sh 2 --log-n 24 26 &&
bash tools/ab_libs.sh 2 --curve bls12_381_g1 --log-n 22 &&
bash tools/ab_libs.sh 2 --curve bls12_381_g2 --log-n 21 &&
bash tools/ab_libs.sh 2 --curve bn254_g2 --log-n 20 &&
GPU_TEST_TIMEOUT=700 bash tools/gpu_check.sh
