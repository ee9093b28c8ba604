#!/bin/bash
# round 5: fold tables for every fixed-base MSM of the Groth16 prover (the
# multi-rank shards and the ungrouped A / B1 / witness + h MSMs too) -- the
# Groth16, dist (sharded proofs), comm and harness files, then the probe:
# default grouped (0) and ungrouped (1), with and without tables (18, 19)
export TMPDIR=/tmp
OUT=gpurun_out/r05ak
mkdir -p $OUT
export TACHYON_MI355X_LIB=$PWD/tachyon_amd/lib_fold2.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_groth16.py tests/test_gpu_dist.py tests/test_gpu_comm.py \
  tests/test_gpu_harness.py tests/test_gpu_msm_fold.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 500 python -u tools/groth16_probe.py --log-n 20 --configs 0,0,0,0 0,0,0,1 0,0,0,18 0,0,0,19 \
  --rounds 3 --reps 10 > $OUT/groth16_fold.jsonl 2>&1
