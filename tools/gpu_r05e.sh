#!/bin/bash
# round 5: A/B of the 2-pass 2^12 x 2^12 NTT plan (12-stage passes, 4096-element
# tiles, 128 KiB LDS) against the 3-pass release plan, tuning build, alternating
# processes; each line checks the round trip
mkdir -p gpurun_out/r05e
export TACHYON_MI355X_LIB=$PWD/tachyon_amd/libtachyon_mi355x_tuning.so
for r in 1 2 3; do
  timeout -k 10 120 python -u tools/tune_ntt.py --log-n 22 24 --reps 20 >> gpurun_out/r05e/ntt_plan_ab.jsonl 2>&1 || exit $?
  TACHYON_NTT_PASS_STAGES=12 TACHYON_NTT_LDS_ELEMS=4096 timeout -k 10 120 python -u tools/tune_ntt.py --log-n 22 24 --reps 20 \
    >> gpurun_out/r05e/ntt_plan_ab.jsonl 2>&1 || exit $?
done
