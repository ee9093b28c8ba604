#!/bin/bash
# round 5: Groth16 fold tables with 3-bit selectors -- the Groth16 parity file,
# then the probe: the default (B2 x8, G1 x4: 0), B2 x16 (10), B2 x4 (6), G1 x2 (32),
# no tables (18)
export TMPDIR=/tmp
OUT=gpurun_out/r05ai
mkdir -p $OUT
export TACHYON_MI355X_LIB=$PWD/tachyon_amd/lib_fold.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_groth16.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 500 python -u tools/groth16_probe.py --log-n 20 --configs 0,0,0,0 0,0,0,10 0,0,0,6 0,0,0,32 0,0,0,18 \
  --rounds 3 --reps 10 > $OUT/groth16_fold.jsonl 2>&1
