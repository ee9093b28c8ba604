#!/bin/bash
# round 4: BLS12-381 28-bit accumulations (G1 + G2 lane pair) parity + A/B, chain-flag check,
# multi-device Groth16, then the NTT probe/PMC.  Stops at the first failing step.
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/$name.log
  return $rc
}
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
[ -z "$SKIP_PARITY" ] && { step bls_tests 500 $P tests/test_gpu_msm.py tests/test_gpu_full_size.py -k "bls" || exit $?
step chain_flags 400 $P tests/test_gpu_msm.py -k "chain_flags" || exit $?; }
step g16_multi 300 $P tests/test_gpu_groth16.py -k "multi_device or devices" || exit $?
step ab_bls 400 python tools/tune_msm.py --curve bls12_381_g1 --log-n 20 22 24 --variants 0 1048576 --rounds 2 || exit $?
step ab_bls_g2 400 python tools/tune_msm.py --curve bls12_381_g2 --log-n 20 22 --variants 0 1048576 --rounds 2 || exit $?
bash tools/ntt_pmc.sh a
