#!/bin/bash
# round 5: fixed-base folding of the Groth16 G2 B query (MsmGpu::fold_bases /
# run_folded) -- fold parity on all four curves, the Groth16 parity files, the
# MSM file, then the Groth16 probe: B2 unfolded (variant 2) / two copies (0,
# the new default) / four copies (6), alternating rounds
export TMPDIR=/tmp
OUT=gpurun_out/r05af
mkdir -p $OUT
export TACHYON_MI355X_LIB=$PWD/tachyon_amd/lib_fold.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm_fold.py tests/test_gpu_groth16.py tests/test_gpu_msm.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/groth16_probe.py --log-n 20 --configs 0,0,0,2 0,0,0,0 0,0,0,6 --rounds 3 --reps 10 \
  > $OUT/groth16_fold.jsonl 2>&1
