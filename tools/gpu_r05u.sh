#!/bin/bash
# round 5: BLS12-381 G1 / G2 window-bit sweep at 2^24 (configs[3]) and BN254 G2
# at 2^20 (the Groth16 B MSM): does the size's plan (c = 20 at 2^24) hold for
# the Fq2 / 381-bit reductions?
OUT=gpurun_out/r05u
mkdir -p $OUT
timeout -k 10 300 python -u tools/tune_msm.py --curve bls12_381_g2 --log-n 24 --c 16 18 19 20 --reps 2 --rounds 2 \
  > $OUT/sweep_bls_g2_2_24.jsonl 2>&1 || exit $?
timeout -k 10 300 python -u tools/tune_msm.py --curve bls12_381_g1 --log-n 24 --c 16 18 19 20 --reps 2 --rounds 2 \
  > $OUT/sweep_bls_g1_2_24.jsonl 2>&1 || exit $?
timeout -k 10 300 python -u tools/tune_msm.py --curve bn254_g2 --log-n 20 --c 14 15 16 17 18 --reps 3 --rounds 2 \
  > $OUT/sweep_bn254_g2_2_20.jsonl 2>&1
