#!/bin/bash
# round 5: precomputed exchange twiddles (tab29) on top of the split plans --
# NTT parity (all NTT tests), then the local-stage probe over splits and
# variants (bit 3 = no table), then a kernel trace of the N = 8 plan
export TMPDIR=/tmp
OUT=gpurun_out/r05q
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_ntt.py tests/test_gpu_ntt_large.py tests/test_gpu_dist.py \
  tests/test_gpu_comm.py -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ntt4_probe.py --log-n 24 --worlds 2 4 8 --variants 0 2 4 8 --rounds 3 \
  --splits 0 -1 > $OUT/ntt4_probe.jsonl 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python tools/ntt4_probe.py --log-n 24 --worlds 8 --variants 0 --rounds 1 --reps 50 --splits -1 > $OUT/trace.log 2>&1
