#!/bin/bash
# Kernel stats of bench.py's Groth16 leg under two library builds:
#   LIB_A=... LIB_B=... tools/trace_groth16.sh
set -e
export TMPDIR=/tmp
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-host-resident --no-sweep --no-non-uniform --no-ntt --bls-log-n 0 --log-n 20"
for tag in A B; do
  var=LIB_$tag
  TACHYON_MI355X_LIB=${!var} timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/g16trace_$tag -o run --output-format csv -- $B > gpurun_out/g16trace_$tag.log 2>&1
done
echo done
