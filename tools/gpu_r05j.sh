#!/bin/bash
# round 5: kernel trace of the four-step NTT's local stages (rank 0 of a 4- and
# an 8-rank 2^24 plan, the fused variant): which kernels the 0.57 / 0.30 ms are
export TMPDIR=/tmp
OUT=gpurun_out/r05j
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python tools/ntt4_probe.py --log-n 24 --worlds 8 --variants 0 --rounds 1 --reps 50 > $OUT/ntt4_w8.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace4 -o run --output-format csv -- \
  python tools/ntt4_probe.py --log-n 24 --worlds 4 --variants 0 --rounds 1 --reps 50 > $OUT/ntt4_w4.log 2>&1
