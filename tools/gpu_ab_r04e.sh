#!/bin/bash
# round 4: LIB_B = the unreduced run start (BN254 G1) + the BN254 G2 29-bit
# lane pair; its MSM / Groth16 parity first, then A/B against LIB_A (HEAD),
# then BN254 G2 window sizes at the Groth16 size (the table is BN254 G1's).
export LIB_A=${LIB_A:-tachyon_amd/ab/lib_a.so} LIB_B=${LIB_B:-tachyon_amd/libtachyon_mi355x.so}
mkdir -p gpurun_out
TACHYON_MI355X_LIB=$LIB_B timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  ${T_MSM-tests/test_gpu_msm.py tests/test_gpu_groth16.py} "tests/test_gpu_ntt.py::test_multi_device_domain_logical" \
  "tests/test_gpu_ntt.py::test_multi_device_domain_refused" > gpurun_out/t_r04e.log 2>&1 &&
bash tools/ab_libs.sh 2 --curve bn254_g1 --log-n 24 26 &&
bash tools/ab_libs.sh 2 --curve bn254_g2 --log-n 20 22 &&
bash tools/gpu_ab_groth16.sh 3 &&
TACHYON_MI355X_LIB=$LIB_B timeout -k 10 200 python tools/tune_msm.py --curve bn254_g2 --log-n 20 --c 12 13 14 15 16 \
  > gpurun_out/tune_g2_2_20.log 2>&1
