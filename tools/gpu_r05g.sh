#!/bin/bash
# round 5: 2-rank gloo rehearsal of bench.py on the one GPU (the N > 1 paths:
# MSM shards combined inside the library over the host-staged process-group
# communicator, the 2-rank NTT on rank 0, the sharded BLS12-381 and Groth16 legs)
mkdir -p gpurun_out/r05g
TACHYON_DIST_BACKEND=gloo timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r05g/bench_gloo_world2.log 2>&1
