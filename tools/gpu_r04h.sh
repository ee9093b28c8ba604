#!/bin/bash
# round 4: rocprofv3 evidence of the final kernels (trace + separate PMC passes),
# then the BLS12-381 G1 / G2 window sizes at the shard sizes 2^21..2^24.
bash tools/profile_round.sh r04b > gpurun_out/profile_r04b.log 2>&1 || exit $?
timeout -k 10 400 python tools/tune_msm.py --curve bls12_381_g1 --log-n 21 22 23 24 --c 15 16 17 18 19 20 \
  > gpurun_out/tune_bls_g1.log 2>&1 &&
timeout -k 10 400 python tools/tune_msm.py --curve bls12_381_g2 --log-n 21 22 23 --c 15 16 17 18 19 \
  > gpurun_out/tune_bls_g2.log 2>&1
