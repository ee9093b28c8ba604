#!/bin/bash
# round 5: A/B of the row-major recode histograms (this tree) against the
# previous commit's library (tachyon_amd/libtachyon_mi355x_old.so), alternating
# processes on one box, plus a kernel trace of each; then the four-step trace
export TMPDIR=/tmp
OUT=gpurun_out/r05l
mkdir -p $OUT
OLD=$PWD/tachyon_amd/libtachyon_mi355x_old.so
for r in 1 2 3; do
  echo "{\"lib\": \"old\", \"round\": $r}" >> $OUT/ab.jsonl
  TACHYON_MI355X_LIB=$OLD timeout -k 10 200 python tools/tune_msm.py --log-n 26 23 20 --reps 5 >> $OUT/ab.jsonl 2>&1 || exit $?
  echo "{\"lib\": \"new\", \"round\": $r}" >> $OUT/ab.jsonl
  timeout -k 10 200 python tools/tune_msm.py --log-n 26 23 20 --reps 5 >> $OUT/ab.jsonl 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_new -o run --output-format csv -- \
  python tools/tune_msm.py --log-n 26 --reps 3 > $OUT/trace_new.log 2>&1 || exit $?
TACHYON_MI355X_LIB=$OLD timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_old -o run --output-format csv -- \
  python tools/tune_msm.py --log-n 26 --reps 3 > $OUT/trace_old.log 2>&1 || exit $?
bash tools/gpu_r05j.sh
