#!/bin/bash
# round 5: PMC passes of the 2^24 NTT, release 3-pass plan vs the 2-pass
# 2^12 x 2^12 plan (tuning build; 12-stage passes, 4096-element tiles): VALU
# and LDS instructions, HBM bytes per transform
export TMPDIR=/tmp
OUT=gpurun_out/r05aa
mkdir -p $OUT
export TACHYON_MI355X_LIB=$PWD/tachyon_amd/libtachyon_mi355x_tuning.so
for plan in 3pass 2pass; do
  if [ $plan = 2pass ]; then export TACHYON_NTT_PASS_STAGES=12 TACHYON_NTT_LDS_ELEMS=4096; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU \
    GRBM_GUI_ACTIVE -d $OUT/valu_$plan -o run --output-format csv -- python tools/tune_ntt.py --log-n 24 --reps 3 \
    > $OUT/valu_$plan.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_$plan -o run --output-format csv -- \
    python tools/tune_ntt.py --log-n 24 --reps 3 > $OUT/fetch_$plan.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write_$plan -o run --output-format csv -- \
    python tools/tune_ntt.py --log-n 24 --reps 3 > $OUT/write_$plan.log 2>&1 || exit $?
done
