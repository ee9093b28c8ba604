#!/bin/bash
# A/B two library builds on the NTT (tools/tune_ntt.py), alternating:
#   LIB_A=... LIB_B=... tools/ab_ntt.sh <rounds> <tune_ntt args...>  -> gpurun_out/ab_ntt.log
set -o pipefail
mkdir -p gpurun_out
R=$1; shift
for i in $(seq 1 $R); do
  for tag in A B; do
    var=LIB_$tag
    echo "== $tag ${!var}" >> gpurun_out/ab_ntt.log
    TACHYON_MI355X_LIB=${!var} timeout -k 10 180 python tools/tune_ntt.py "$@" >> gpurun_out/ab_ntt.log 2>&1 || exit $?
  done
done
