#!/bin/bash
# Alternate several library builds on one box: tools/ab_multi.sh <rounds> "<lib> <lib> ..." <tune args...>
# Writes gpurun_out/ab_multi.log; stops at the first failing run.
set -o pipefail
mkdir -p gpurun_out
R=$1; LIBS=$2; shift 2
for i in $(seq 1 $R); do
  for lib in $LIBS; do
    echo "== $lib" >> gpurun_out/ab_multi.log
    TACHYON_MI355X_LIB=$lib timeout -k 10 180 python tools/tune_msm.py "$@" >> gpurun_out/ab_multi.log 2>&1 || exit $?
  done
done
