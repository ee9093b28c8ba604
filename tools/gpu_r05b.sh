#!/bin/bash
# round 5: library communicators (RCCL world 1, host-staged world 2), the dist
# tests, the four-step variants (parity, then the local-stage A/B), and the
# window-size sweep at the multi-GPU shard sizes
mkdir -p gpurun_out/r05b
timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_comm.py tests/test_gpu_dist.py "tests/test_gpu_ntt.py::test_four_step_simulated_ranks" \
  tests/test_gpu_ntt_large.py::test_four_step_2_25 tests/test_gpu_groth16.py "tests/test_gpu_ntt.py::test_multi_device_domain_logical" \
  "tests/test_gpu_ntt.py::test_multi_device_domain_refused" tests/test_gpu_ntt_large.py::test_multi_device_domain_2_25_logical \
  > gpurun_out/r05b/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ntt4_probe.py --log-n 24 --worlds 2 4 8 --variants 0 1 2 3 --rounds 3 \
  > gpurun_out/r05b/ntt4_probe.jsonl 2>&1 || exit $?
timeout -k 10 300 python -u tools/groth16_probe.py --log-n 20 --rounds 3 \
  --configs 0,0,0,1 0,0,0 0,0,17 0,0,15 16,0,17 17,0,0 > gpurun_out/r05b/groth16_probe.jsonl 2>&1 || exit $?

