#!/bin/bash
# A/B two builds of the library on one GPU box (alternating, to cancel drift):
#   tools/ab_libs.sh <rounds> <tune args...>   with LIB_A / LIB_B paths in the env
# Writes gpurun_out/ab.log; stops at the first failing run.
set -o pipefail
mkdir -p gpurun_out
R=$1; shift
for i in $(seq 1 $R); do
  for tag in A B; do
    var=LIB_$tag
    echo "== $tag ${!var}" >> gpurun_out/ab.log
    TACHYON_MI355X_LIB=${!var} timeout -k 10 180 python tools/tune_msm.py "$@" >> gpurun_out/ab.log 2>&1 || exit $?
  done
done
