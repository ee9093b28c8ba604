#!/bin/bash
# round 4: the 29-bit NTT passes as the default up to 2^20 -- parity (NTT,
# distributed four-step on one GPU, Groth16, KZG), small-size A/B, Groth16 A/B
export LIB_A=${LIB_A:-tachyon_amd/ab/lib_a.so} LIB_B=${LIB_B:-tachyon_amd/libtachyon_mi355x.so}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_ntt.py tests/test_gpu_groth16.py tests/test_gpu_kzg.py tests/test_gpu_dist.py > gpurun_out/t_ntt29.log 2>&1 &&
for lg in 16 18 20 21; do
  timeout -k 10 200 python tools/ntt_probe.py --log-n $lg --reps 50 --variants 0,1 --rounds 4 >> gpurun_out/ntt_ab_small.log 2>&1 || exit $?
done &&
bash tools/gpu_ab_groth16.sh 3
