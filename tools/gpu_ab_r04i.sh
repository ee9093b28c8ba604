#!/bin/bash
# round 4: Groth16 with the A MSM after B2 on the G2 stream (TACHYON_G16_A_AFTER_B2,
# A/B in alternation, parity first) and the BLS12-381 window rule (c = 16 instead of 17)
mkdir -p gpurun_out
TACHYON_G16_A_AFTER_B2=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_groth16.py > gpurun_out/t_g16_order.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_msm.py \
  > gpurun_out/t_msm_wrule.log 2>&1 || exit $?
for i in 1 2 3; do
  for v in 0 1; do
    TACHYON_G16_A_AFTER_B2=$v timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-resident \
      --no-sweep --no-non-uniform --no-ntt --bls-log-n 0 --log-n 20 > gpurun_out/g16_o$v.json 2>/dev/null || exit 1
    tail -n 1 gpurun_out/g16_o$v.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('a_after_b2=$v', d['groth16']['ms_per_proof'], d['groth16']['phase_ms'])" >> gpurun_out/ab_g16_order.log
  done
done
timeout -k 10 300 python tools/tune_msm.py --curve bls12_381_g1 --log-n 22 23 > gpurun_out/bls_wrule.log 2>&1 &&
timeout -k 10 300 python tools/tune_msm.py --curve bls12_381_g2 --log-n 22 23 >> gpurun_out/bls_wrule.log 2>&1
