#!/bin/bash
# round 5: Groth16 fold tables, four vs eight copies (variant bits 1-2 / 3-4 =
# 3: eight) -- the Groth16 parity file, then the probe: both four (0, the
# default), B2 eight (6), G1 eight (24), both eight (30)
export TMPDIR=/tmp
OUT=gpurun_out/r05ah
mkdir -p $OUT
export TACHYON_MI355X_LIB=$PWD/tachyon_amd/lib_fold.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_groth16.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 500 python -u tools/groth16_probe.py --log-n 20 --configs 0,0,0,0 0,0,0,6 0,0,0,24 0,0,0,30 \
  --rounds 3 --reps 10 > $OUT/groth16_fold.jsonl 2>&1
