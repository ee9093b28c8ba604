#!/bin/bash
# round 5: 4-rank gloo rehearsal of bench.py on the one GPU with the hybrid MSM
# partition (2 point groups x 2 window groups, c = 19: the plan --msm-split
# auto runs from 8 GPUs) -- consistent_with_1gpu checks the combined MSM
mkdir -p gpurun_out/r05i
TACHYON_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 4 --steps 2 --warmup 1 --no-cpu-baseline \
  --msm-split hybrid --window-groups 2 > gpurun_out/r05i/bench_gloo_world4_hybrid.log 2>&1
