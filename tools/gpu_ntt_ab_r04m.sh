#!/bin/bash
# round 4: NTT 32-bit vs 29-bit passes (domain variants 0 / 1 / 3), more rounds, 2^20..2^24
mkdir -p gpurun_out
for lg in 24 22 20; do
  timeout -k 10 300 python tools/ntt_probe.py --log-n $lg --reps 20 --variants 0,1,3 --rounds 6 >> gpurun_out/ntt_ab_r04m.log 2>&1 || exit $?
done
