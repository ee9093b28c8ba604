#!/bin/bash
# round 4: the batched MSM's window size -- batch ms over a sweep of c (0 = the shipped rule)
mkdir -p gpurun_out
timeout -k 10 400 python tools/batch_probe.py --log-len 10 12 14 16 --count 8 32 128 --reps 3 \
  --c 0 8 9 10 11 12 13 14 15 16 > gpurun_out/batch_probe3.log 2>&1
