#!/bin/bash
# round 5: onesweep tile shapes A/B at 2^26 (tuning build: TACHYON_ONESWEEP_CFG
# 0 = 1024 x 8 (release), 3 = 1024 x 12, 4 = 1024 x 16, 5 = 512 x 16), 3 rounds
OUT=gpurun_out/r05y
mkdir -p $OUT
export TACHYON_MI355X_LIB=$PWD/tachyon_amd/libtachyon_mi355x_tuning.so
for r in 1 2 3; do
  for cfg in 0 3 4 5; do
    echo "{\"onesweep_cfg\": $cfg, \"round\": $r}" >> $OUT/ab.jsonl
    TACHYON_ONESWEEP_CFG=$cfg timeout -k 10 200 python tools/tune_msm.py --log-n 26 23 --reps 3 >> $OUT/ab.jsonl 2>&1 || exit $?
  done
done
