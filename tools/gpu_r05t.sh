#!/bin/bash
# round 5: Groth16 2^20 proof-time series (12 proofs per configuration, 3
# rounds) with the round's final MSM code
OUT=gpurun_out/r05t
mkdir -p $OUT
timeout -k 10 600 python -u tools/groth16_probe.py --log-n 20 --configs 0,0,0 0,0,14 0,0,16 --rounds 3 --reps 12 \
  > $OUT/groth16_series.jsonl 2>&1
