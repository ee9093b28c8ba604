#!/bin/bash
# round 5: running-sum segment length of the BLS12-381 G1 window sums
# (TACHYON_MSM_SEG, tuning build) at 2^24 and 2^22: reduction 5.6 ms of 41.8
# at 2^24 with the G1 rule's L = 64
export TMPDIR=/tmp
OUT=gpurun_out/r05aq
mkdir -p $OUT
export TACHYON_MI355X_LIB=$PWD/tachyon_amd/libtachyon_mi355x_tuning.so
for r in 1 2; do
  for seg in 64 128 32; do
    echo "{\"seg\": $seg, \"round\": $r}" >> $OUT/seg.jsonl
    TACHYON_MSM_SEG=$seg timeout -k 10 300 python tools/tune_msm.py --curve bls12_381_g1 --log-n 24 22 --reps 2 \
      >> $OUT/seg.jsonl 2>&1 || exit $?
  done
done
