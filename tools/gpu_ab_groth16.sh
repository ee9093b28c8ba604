#!/bin/bash
# A/B the Groth16 leg of bench.py between two library builds (alternating, one box):
#   LIB_A=... LIB_B=... tools/gpu_ab_groth16.sh <rounds>
set -o pipefail
mkdir -p gpurun_out
for i in $(seq 1 $1); do
  for tag in A B; do
    var=LIB_$tag
    TACHYON_MI355X_LIB=${!var} timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-host-resident \
      --no-sweep --no-non-uniform --no-ntt --bls-log-n 0 --log-n 20 > gpurun_out/g16_$tag.json 2>/dev/null || exit 1
    tail -n 1 gpurun_out/g16_$tag.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['groth16']['ms_per_proof'], d['groth16']['phase_ms'])" >> gpurun_out/ab_g16.log
  done
done
