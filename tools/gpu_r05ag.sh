#!/bin/bash
# round 5: fixed-base fold tables of both Groth16 MSM streams (the G2 B query,
# run_folded; the grouped A + witness + h G1 MSM, run_groups_folded) -- fold,
# Groth16, MSM and KZG parity, then the Groth16 probe: no folds (10), B2 only
# (8), G1 only (2), both four copies (0, the new default), both two (20)
export TMPDIR=/tmp
OUT=gpurun_out/r05ag
mkdir -p $OUT
export TACHYON_MI355X_LIB=$PWD/tachyon_amd/lib_fold.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm_fold.py tests/test_gpu_groth16.py tests/test_gpu_msm.py \
  tests/test_gpu_kzg.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 500 python -u tools/groth16_probe.py --log-n 20 --configs 0,0,0,10 0,0,0,8 0,0,0,2 0,0,0,0 0,0,0,20 \
  --rounds 3 --reps 10 > $OUT/groth16_fold.jsonl 2>&1
