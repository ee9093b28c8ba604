#!/bin/bash
# round 5: gloo rehearsals of the multi-rank bench on one GPU (fold tables in the sharded Groth16 proofs) with the final
# plan table (BN254 G1 hybrid at N = 8 only; BLS12-381 G1 point shards; G2
# hybrid at N = 4 and 8): 2 and 4 ranks, default arguments otherwise
export TMPDIR=/tmp
OUT=gpurun_out/r05ap
mkdir -p $OUT
TACHYON_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29593 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline \
  > $OUT/bench_gloo_world2.log 2>&1 || exit $?
TACHYON_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29594 bench.py --gpus 4 --steps 2 --warmup 1 --no-cpu-baseline \
  > $OUT/bench_gloo_world4.log 2>&1
