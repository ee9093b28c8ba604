#!/bin/bash
# rocprofv3 evidence for one round: kernel trace (+stats) of the bench command,
# then separate PMC passes (FETCH_SIZE / WRITE_SIZE / VALU counters), as the
# MI355X_MICROARCH.md HBM/rocprofv3 section prescribes (one counter group per pass).
#   ./tools/profile_round.sh r01 [bench args...]
set -e
TAG=${1:-r01}; shift || true
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline $*"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/bench_under_trace.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > $OUT/write.log 2>&1
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/valu -o run --output-format csv -- $B > $OUT/valu.log 2>&1
python tools/summarize_profile.py $OUT > $OUT/summary.md
echo done
