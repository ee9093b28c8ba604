#!/bin/bash
# Per-kernel times of two library builds on one box: a rocprofv3 kernel trace
# of the same tune_msm run under each (LIB_A / LIB_B in the env).
#   tools/ab_kernels.sh <tune args...>   -> gpurun_out/abk_{A,B}/ + abk.txt
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for tag in A B; do
  var=LIB_$tag
  TACHYON_MI355X_LIB=${!var} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abk_$tag -o run \
    --output-format csv -- python tools/tune_msm.py "$@" > gpurun_out/abk_$tag.log 2>&1
  echo "== $tag ${!var}" >> gpurun_out/abk.txt
  cat gpurun_out/abk_$tag/*/run_kernel_stats.csv gpurun_out/abk_$tag/run_kernel_stats.csv 2>/dev/null \
    | cut -d, -f1-6 | head -25 >> gpurun_out/abk.txt || true
done
