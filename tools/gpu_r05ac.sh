#!/bin/bash
# round 5: running-sum segment length of the BN254 G1 window sums
# (TACHYON_MSM_SEG, tuning build) at 2^23..2^26 -- at 2^26 the default L = 64
# gives 106 K segment threads (1.6 waves per SIMD) for window_segment29_kernel
export TMPDIR=/tmp
OUT=gpurun_out/r05ac
mkdir -p $OUT
export TACHYON_MI355X_LIB=$PWD/tachyon_amd/libtachyon_mi355x_tuning.so
for r in 1 2; do
  for seg in 64 32 16 128; do
    echo "{\"seg\": $seg, \"round\": $r}" >> $OUT/seg.jsonl
    TACHYON_MSM_SEG=$seg timeout -k 10 200 python tools/tune_msm.py --log-n 26 25 24 23 --reps 3 >> $OUT/seg.jsonl 2>&1 || exit $?
  done
done
