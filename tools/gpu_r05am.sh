#!/bin/bash
# round 5: running-sum segment length of the G2 window sums (TACHYON_MSM_SEG,
# tuning build): BLS12-381 G2 2^24 (reduction 13.7 ms of 107 at c = 20) and
# BN254 G2 2^22, L = 64 (the plan) / 32 / 16 / 128, 2 rounds
export TMPDIR=/tmp
OUT=gpurun_out/r05am
mkdir -p $OUT
export TACHYON_MI355X_LIB=$PWD/tachyon_amd/libtachyon_mi355x_tuning.so
for r in 1 2; do
  for seg in 64 32 16 128; do
    echo "{\"seg\": $seg, \"round\": $r}" >> $OUT/seg.jsonl
    TACHYON_MSM_SEG=$seg timeout -k 10 300 python tools/tune_msm.py --curve bls12_381_g2 --log-n 24 --reps 2 \
      >> $OUT/seg.jsonl 2>&1 || exit $?
    TACHYON_MSM_SEG=$seg timeout -k 10 300 python tools/tune_msm.py --curve bn254_g2 --log-n 22 --reps 2 \
      >> $OUT/seg.jsonl 2>&1 || exit $?
  done
done
