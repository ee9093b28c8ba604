#!/bin/bash
# round 5: the hybrid partition for BLS12-381 G1 / G2 at 2^24 (BASELINE
# configs[3]): slowest-rank times of P point groups x Q window groups
OUT=gpurun_out/r05m
mkdir -p $OUT
timeout -k 10 400 python -u tools/split_probe.py --curve bls12_381_g1 --log-n 24 --worlds 8 4 --hybrid \
  --hybrid-c 15 16 17 19 --reps 3 > $OUT/hybrid_bls_g1.jsonl 2>&1 || exit $?
timeout -k 10 600 python -u tools/split_probe.py --curve bls12_381_g2 --log-n 24 --worlds 8 4 --hybrid \
  --hybrid-c 15 16 17 19 --reps 3 > $OUT/hybrid_bls_g2.jsonl 2>&1
