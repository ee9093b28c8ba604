#!/bin/bash
# round 5: batch-affine vs XYZZ madd in registers: the
# probe's timing rows, then one PMC pass for VALU / LDS instructions per kernel
OUT=gpurun_out/r05h
mkdir -p $OUT
timeout -k 10 300 ./tachyon_amd/bin/batch_affine_probe 4 > $OUT/batch_affine_probe.jsonl 2> $OUT/batch_affine_probe.err || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES -d $OUT/pmc -o run \
  --output-format csv -- ./tachyon_amd/bin/batch_affine_probe 1 > $OUT/pmc.log 2>&1
