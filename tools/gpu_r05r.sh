#!/bin/bash
# round 5: profile + default bench line of the current library, then a 4-rank
# gloo rehearsal of the default bench (four-step NTT on the new exchange layout,
# BLS12-381 hybrid plans)
bash tools/profile_round.sh r05r || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_full_r05r.log 2>&1 || exit $?
mkdir -p gpurun_out/r05r
TACHYON_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29591 bench.py --gpus 4 --steps 2 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r05r/bench_gloo_world4_auto.log 2>&1
