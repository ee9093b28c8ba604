#!/bin/bash
# round 5: window-size sweep at the per-rank shard sizes of the multi-GPU
# configs (BN254 G1 2^26 / N = 2^23..2^25; BLS12-381 G1 / G2 2^24 / N =
# 2^21..2^23), 2 rounds x 5 reps, HIP-event phases per run
mkdir -p gpurun_out/r05c
timeout -k 10 400 python -u tools/tune_msm.py --curve bn254_g1 --log-n 23 24 25 --c 16 17 19 20 22 --reps 5 --rounds 2 \
  > gpurun_out/r05c/sweep_bn254_g1.jsonl 2>&1 || exit $?
timeout -k 10 300 python -u tools/tune_msm.py --curve bls12_381_g1 --log-n 21 22 23 --c 14 15 16 18 19 20 --reps 3 --rounds 2 \
  > gpurun_out/r05c/sweep_bls12_381_g1.jsonl 2>&1 || exit $?
timeout -k 10 400 python -u tools/tune_msm.py --curve bls12_381_g2 --log-n 21 22 23 --c 14 15 16 18 19 --reps 3 --rounds 1 \
  > gpurun_out/r05c/sweep_bls12_381_g2.jsonl 2>&1 || exit $?
timeout -k 10 400 python -u tools/split_probe.py --log-n 26 --worlds 2 4 8 --hybrid --hybrid-c 17 19 20 --reps 3 \
  > gpurun_out/r05c/hybrid_split_probe.jsonl 2>&1
