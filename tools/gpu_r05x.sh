#!/bin/bash
# round 5: MSM parity with the two-level window sums back to an A/B variant
# (edge cases through bit 23 on every curve), Groth16 back on the one-level sums
OUT=gpurun_out/r05x
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_groth16.py -m gpu -x -q \
  --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/groth16_probe.py --log-n 20 --configs 0,0,0 --rounds 2 --reps 12 > $OUT/groth16.jsonl 2>&1
