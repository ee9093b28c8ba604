#!/bin/bash
# round 5: two-level G2 window sums -- G2 parity (MSM, BLS12-381, Groth16, KZG
# files), then A/B against the one-level kernel (variant bit 23) on BLS12-381
# G2 2^24 and BN254 G2 2^20, alternating in one process per size
OUT=gpurun_out/r05w
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_full_size.py tests/test_gpu_groth16.py \
  -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/tune_msm.py --curve bls12_381_g2 --log-n 24 --variants 0 8388608 --reps 2 --rounds 3 \
  > $OUT/ab_bls_g2_2_24.jsonl 2>&1 || exit $?
timeout -k 10 300 python -u tools/tune_msm.py --curve bn254_g2 --log-n 20 22 --variants 0 8388608 --reps 3 --rounds 3 \
  > $OUT/ab_bn254_g2.jsonl 2>&1 || exit $?
timeout -k 10 300 python -u tools/groth16_probe.py --log-n 20 --configs 0,0,0 --rounds 2 --reps 12 > $OUT/groth16.jsonl 2>&1
