#!/bin/bash
# round 5: the new large-domain NTT tests and the touched Groth16 / KZG tests,
# then the default bench line (first measurement of the round)
mkdir -p gpurun_out/r05a
timeout -k 10 700 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_gpu_ntt_large.py tests/test_gpu_kzg.py "tests/test_gpu_groth16.py::test_multi_device_prover" tests/test_gpu_harness.py \
  > gpurun_out/r05a/tests.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/r05a/bench.log 2>&1
