#!/bin/bash
# round 5: full-size 2^24 four-step on the bench's split (4 and 8 simulated
# ranks) + the in-register madd ceiling at two launch lengths (13 vs 80 ms:
# does the clock under a long launch set the accumulation's VALU gap?)
OUT=gpurun_out/r05s
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_ntt_large.py -m gpu -x -q -k "split or 2_25" \
  --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
for r in 4 20 4 20; do
  timeout -k 10 120 ./tachyon_amd/bin/batch_affine_probe $r > $OUT/madd_len_$r.jsonl 2>&1 || exit $?
  grep madd_reg $OUT/madd_len_$r.jsonl >> $OUT/madd_ceiling_by_length.jsonl
done
