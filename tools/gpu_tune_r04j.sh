#!/bin/bash
# accumulation chunk K (set_variant bits 0-1: x2, x4, /2) at the Groth16 MSM sizes
mkdir -p gpurun_out
timeout -k 10 300 python tools/tune_msm.py --curve bn254_g2 --log-n 20 --variants 0 1 2 3 --rounds 2 > gpurun_out/tune_k_g2.log 2>&1 &&
timeout -k 10 300 python tools/tune_msm.py --curve bn254_g1 --log-n 20 21 --variants 0 1 2 3 --rounds 2 > gpurun_out/tune_k_g1.log 2>&1
