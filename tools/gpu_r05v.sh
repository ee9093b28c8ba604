#!/bin/bash
# round 5: kernel trace of the BLS12-381 G2 2^24 MSM (its bucket reduction is
# 13.9 ms of 108): which reduction kernels, how long, and their registers
export TMPDIR=/tmp
OUT=gpurun_out/r05v
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python tools/tune_msm.py --curve bls12_381_g2 --log-n 24 --reps 2 > $OUT/trace.log 2>&1
