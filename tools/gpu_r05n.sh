#!/bin/bash
# round 5: the third-place count copies in recode_hist_kernel -- MSM parity,
# A/B against the previous commit's library (alternating processes), then a
# 4-rank gloo rehearsal of the default bench (auto partition: BN254 point
# shards, BLS12-381 G1 / G2 hybrid at N = 4)
export TMPDIR=/tmp
OUT=gpurun_out/r05n
mkdir -p $OUT
OLD=$PWD/tachyon_amd/libtachyon_mi355x_old.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_full_size.py -m gpu -x -q \
  --timeout 500 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
for r in 1 2 3; do
  echo "{\"lib\": \"old\", \"round\": $r}" >> $OUT/ab.jsonl
  TACHYON_MI355X_LIB=$OLD timeout -k 10 200 python tools/tune_msm.py --log-n 26 23 20 --reps 5 >> $OUT/ab.jsonl 2>&1 || exit $?
  echo "{\"lib\": \"new\", \"round\": $r}" >> $OUT/ab.jsonl
  timeout -k 10 200 python tools/tune_msm.py --log-n 26 23 20 --reps 5 >> $OUT/ab.jsonl 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_new -o run --output-format csv -- \
  python tools/tune_msm.py --log-n 26 23 20 --reps 3 > $OUT/trace_new.log 2>&1 || exit $?
TACHYON_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29581 bench.py --gpus 4 --steps 2 --warmup 1 --no-cpu-baseline \
  > $OUT/bench_gloo_world4_auto.log 2>&1
