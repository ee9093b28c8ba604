#!/bin/bash
# round 4: Groth16 with one recode + sort shared by the A and B-in-G2 MSMs
# (parity, then A/B against LIB_A), and the accumulation chunk K at 2^18..2^25
# (set_variant bits 0-1: K x2 / x4)
export LIB_A=${LIB_A:-tachyon_amd/ab/lib_a.so} LIB_B=${LIB_B:-tachyon_amd/libtachyon_mi355x.so}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_groth16.py > gpurun_out/t_g16_share.log 2>&1 &&
bash tools/gpu_ab_groth16.sh 3 &&
timeout -k 10 400 python tools/tune_msm.py --curve bn254_g1 --log-n 18 19 20 21 22 23 24 25 --variants 0 1 2 --rounds 2 \
  > gpurun_out/tune_k_sweep.log 2>&1
