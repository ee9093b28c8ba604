#!/bin/bash
# round 5: G2 window segment sums in two passes (set_variant bit 24: suffix
# sums stored, then summed, then the fix-ups) -- G2 golden / edge-case parity
# with the bit, then one-pass vs two-pass at segment lengths L = 32 / 64 / 128
# (tuning build, TACHYON_MSM_SEG) on BLS12-381 G2 2^24 and BN254 G2 2^22,
# alternating in one process per L
export TMPDIR=/tmp
OUT=gpurun_out/r05an
mkdir -p $OUT
export TACHYON_MI355X_LIB=$PWD/tachyon_amd/lib_rsum_t.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "g2 or reduction" > $OUT/tests.log 2>&1 || exit $?
for seg in 64 128 32; do
  echo "{\"seg\": $seg}" >> $OUT/ab.jsonl
  TACHYON_MSM_SEG=$seg timeout -k 10 400 python -u tools/tune_msm.py --curve bls12_381_g2 --log-n 24 \
    --variants 0 16777216 --reps 2 --rounds 2 >> $OUT/ab.jsonl 2>&1 || exit $?
  TACHYON_MSM_SEG=$seg timeout -k 10 300 python -u tools/tune_msm.py --curve bn254_g2 --log-n 22 \
    --variants 0 16777216 --reps 2 --rounds 2 >> $OUT/ab.jsonl 2>&1 || exit $?
done
