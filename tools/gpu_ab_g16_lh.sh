#!/bin/bash
# Groth16: the l + h MSM on a third stream (TACHYON_G16_LH_STREAM=1) -- parity, then A/B in alternation
mkdir -p gpurun_out
TACHYON_G16_LH_STREAM=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_groth16.py > gpurun_out/t_g16_lh.log 2>&1 || exit $?
for i in 1 2 3; do
  for v in 0 1; do
    TACHYON_G16_LH_STREAM=$v timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-host-resident \
      --no-sweep --no-non-uniform --no-ntt --bls-log-n 0 --log-n 20 > gpurun_out/g16_lh$v.json 2>/dev/null || exit 1
    tail -n 1 gpurun_out/g16_lh$v.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lh_stream=$v', d['groth16']['ms_per_proof'], d['groth16']['phase_ms'])" >> gpurun_out/ab_g16_lh.log
  done
done
