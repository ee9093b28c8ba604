#!/bin/bash
# round 5: window bits of the BLS12-381 2^24 MSMs (the bench's BLS leg; the
# plan gives c = 20, W = 13): G2 and G1 at c = 17..21, 2 alternating rounds
export TMPDIR=/tmp
OUT=gpurun_out/r05al
mkdir -p $OUT
timeout -k 10 600 python -u tools/tune_msm.py --curve bls12_381_g2 --log-n 24 --c 20 18 19 17 21 --reps 2 --rounds 2 \
  > $OUT/bls_g2_c.jsonl 2>&1 || exit $?
timeout -k 10 400 python -u tools/tune_msm.py --curve bls12_381_g1 --log-n 24 --c 20 18 19 17 21 --reps 2 --rounds 2 \
  > $OUT/bls_g1_c.jsonl 2>&1
