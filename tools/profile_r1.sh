#!/bin/bash
# rocprofv3 kernel trace + PMC passes of bench.py (MSM 2^26 + NTT 2^24).
set -e
export TMPDIR=/tmp
OUT=gpurun_out/prof_r1
mkdir -p $OUT
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/valu -o run --output-format csv -- $B > $OUT/valu.log 2>&1
echo done
