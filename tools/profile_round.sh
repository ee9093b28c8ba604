#!/bin/bash
# rocprofv3 evidence for one round, run on the GPU box:
#   ./tools/profile_round.sh r02 [bench args...]
# 1. kernel trace + stats of the bench command;
# 2. separate PMC passes (FETCH_SIZE, WRITE_SIZE, VALU counters), one counter
#    group per pass as MI355X_MICROARCH.md's HBM/rocprofv3 section prescribes;
# 3. summary.md + pmc_traffic.json (per-dispatch HBM bytes that bench.py puts in
#    its roofline "traffic" field) + kernel_stats.csv in gpurun_out/prof_<tag>/publish
#    (gpurun merges gpurun_out/ back; copy that directory to profiles/<tag>/).
set -e
TAG=${1:-r01}; shift || true
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-resident --no-sweep --groth16-log-n 0 --bls-log-n 0 $*"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/bench_under_trace.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > $OUT/write.log 2>&1
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/valu -o run --output-format csv -- $B > $OUT/valu.log 2>&1
python tools/summarize_profile.py $OUT > $OUT/summary.md
P=$OUT/publish
mkdir -p $P
cp $OUT/summary.md $OUT/pmc_traffic.json $P/
cp $OUT/trace/run_kernel_stats.csv $P/kernel_stats.csv
grep "^{\"metric\"" $OUT/bench_under_trace.log | tail -n 1 > $P/bench_under_trace.json
echo done
