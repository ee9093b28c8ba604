#!/bin/bash
# round 5: the four-step local-stage A/B and the Groth16 grouped-MSM / window probe
mkdir -p gpurun_out/r05b
timeout -k 10 300 python -u tools/ntt4_probe.py --log-n 24 --worlds 2 4 8 --variants 0 1 2 3 --rounds 3 \
  > gpurun_out/r05b/ntt4_probe.jsonl 2>&1 || exit $?
timeout -k 10 300 python -u tools/groth16_probe.py --log-n 20 --rounds 3 \
  --configs 0,0,0,1 0,0,0 0,0,17 0,0,15 16,0,17 17,0,0 > gpurun_out/r05b/groth16_probe.jsonl 2>&1 || exit $?
bash tools/gpu_r05c.sh
