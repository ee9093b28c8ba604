#!/bin/bash
# GPU box: A/B of the in-tree library (A) against LIB_B on the BN254 G1 MSM
# (2^24, 2^26) and the BN254 G2 MSM (2^20).
export LIB_A=tachyon_amd/libtachyon_mi355x.so
mkdir -p gpurun_out
bash tools/ab_libs.sh 2 --log-n 24 26 &&
bash tools/ab_libs.sh 2 --curve bn254_g2 --log-n 20
