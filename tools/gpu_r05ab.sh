#!/bin/bash
# round 5: the recode's per-scalar work -- (a) from_mont as a bare Montgomery
# reduction (64 instead of 128 v_mad_u64_u32 per scalar in each recode pass),
# (b) plus compile-time window widths (16 / 17 / 20: one bit-field extract
# per window instead of N funnel shifts).  Parity of everything that converts
# out of Montgomery form on the device with (b), then an A/B of release / (a) /
# (b) in alternating processes, Groth16, and a kernel trace per library.
export TMPDIR=/tmp
OUT=gpurun_out/r05ab
mkdir -p $OUT
REL=$PWD/tachyon_amd/libtachyon_mi355x.so
A=$PWD/tachyon_amd/lib_redc.so
B=$PWD/tachyon_amd/lib_redc_c.so
TACHYON_MI355X_LIB=$B timeout -k 10 900 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_field_ec.py \
  tests/test_gpu_ntt.py tests/test_gpu_groth16.py tests/test_gpu_kzg.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/tests.log 2>&1 || exit $?
for r in 1 2 3; do
  for lib in rel redc redc_c; do
    L=$REL; [ $lib = redc ] && L=$A; [ $lib = redc_c ] && L=$B
    echo "{\"lib\": \"$lib\", \"round\": $r}" >> $OUT/ab.jsonl
    TACHYON_MI355X_LIB=$L timeout -k 10 200 python tools/tune_msm.py --log-n 26 23 20 --reps 5 >> $OUT/ab.jsonl 2>&1 || exit $?
  done
done
for lib in rel redc_c; do
  L=$REL; [ $lib = redc_c ] && L=$B
  TACHYON_MI355X_LIB=$L timeout -k 10 200 python tools/groth16_probe.py --log-n 20 --configs 0,0,0 --rounds 2 --reps 12 \
    > $OUT/groth16_$lib.jsonl 2>&1 || exit $?
  TACHYON_MI355X_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$lib -o run --output-format csv -- \
    python tools/tune_msm.py --log-n 26 --reps 3 > $OUT/trace_$lib.log 2>&1 || exit $?
done
