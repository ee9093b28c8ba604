#!/bin/bash
# round 5: row-major recode histograms -- MSM / KZG / Groth16 parity, then the
# default bench's MSM phases (recode before: 5.09 ms at 2^26, profiles/r05f)
OUT=gpurun_out/r05k
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_full_size.py tests/test_gpu_kzg.py \
  tests/test_gpu_groth16.py -m gpu -x -q --timeout 600 --timeout-method thread \
  > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-resident --no-sweep > $OUT/bench.log 2>&1
