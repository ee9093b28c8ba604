#!/bin/bash
# round 4: BLS12-381 G1 28-bit accumulation parity + A/B, multi-device Groth16, then the NTT probe/PMC
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_full_size.py -x -q -k "bls12_381_g1 or bls" --timeout 300 --timeout-method thread > gpurun_out/bls_tests.log 2>&1
rc=$?; echo "bls tests rc=$rc" >> gpurun_out/bls_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_groth16.py -x -q -k "multi_device or devices" --timeout 200 --timeout-method thread > gpurun_out/g16_multi_tests.log 2>&1
rc=$?; echo "g16 multi rc=$rc" >> gpurun_out/g16_multi_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python tools/tune_msm.py --curve bls12_381_g1 --log-n 20 22 24 --variants 0 1048576 --rounds 2 > gpurun_out/ab_bls_g1_acc28.log 2>&1 || exit $?
bash tools/ntt_pmc.sh a
