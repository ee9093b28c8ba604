#!/bin/bash
# Three-way A/B of library builds (alternating, one box):  tools/gpu_ab3.sh <rounds> <libs...> -- <tune args>
set -o pipefail
mkdir -p gpurun_out
R=$1; shift
LIBS=()
while [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
shift
for i in $(seq 1 $R); do
  for L in "${LIBS[@]}"; do
    echo "== $L" >> gpurun_out/ab3.log
    TACHYON_MI355X_LIB=$L timeout -k 10 180 python tools/tune_msm.py "$@" >> gpurun_out/ab3.log 2>&1 || exit $?
  done
done
