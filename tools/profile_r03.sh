#!/bin/bash
# Round-3 rocprofv3 evidence, run on the GPU box:  ./tools/profile_r03.sh <tag>
#  1. kernel trace + stats of the bench command (BN254 G1 2^26 MSM + 2^24 NTT);
#  2. separate PMC passes of the same command, one counter group each
#     (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass):
#     fetch, write, valu (instruction mix + cycles), occ (resident waves:
#     MeanOccupancyPerCU = accumulated SQ_LEVEL_WAVES / GUI cycles / CUs);
#  3. trace + valu passes of a BLS12-381 G2 2^22 MSM (lane-pair kernels);
#  4. valu pass of the in-register mixed-addition microbenchmark
#     (tools/microbench/madd_rates: the accumulation's VALU ceiling and clock);
#  5. summary.md + pmc_r03.json (tools/summarize_r03.py) and summary_traffic.md +
#     pmc_traffic.json (tools/summarize_profile.py: bench.py's roofline traffic).
# Every pass under its own timeout; the first failure ends the script.
set -e
TAG=${1:-r03}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-resident --no-sweep --no-non-uniform --groth16-log-n 0 --bls-log-n 0"
VALU="SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
OCC="MeanOccupancyPerCU SQ_WAVES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/bench_under_trace.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > $OUT/write.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc $VALU -d $OUT/valu -o run --output-format csv -- $B > $OUT/valu.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc $OCC -d $OUT/occ -o run --output-format csv -- $B > $OUT/occ.log 2>&1
G2="python tools/tune_msm.py --curve bls12_381_g2 --log-n 22 --reps 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/g2_trace -o run --output-format csv -- $G2 > $OUT/g2.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc $VALU -d $OUT/g2_valu -o run --output-format csv -- $G2 >> $OUT/g2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc $VALU -d $OUT/micro_valu -o run --output-format csv -- ./tools/microbench/madd_rates > $OUT/micro.log 2>&1
python tools/summarize_r03.py $OUT > $OUT/summary.md
python tools/summarize_profile.py $OUT > $OUT/summary_traffic.md
P=$OUT/publish
mkdir -p $P
cp $OUT/summary.md $OUT/summary_traffic.md $OUT/pmc_traffic.json $OUT/pmc_r03.json $OUT/micro.log $P/
cp $OUT/trace/run_kernel_stats.csv $P/kernel_stats.csv
cp $OUT/g2_trace/run_kernel_stats.csv $P/kernel_stats_bls12_381_g2_2_22.csv
grep '^{' $OUT/bench_under_trace.log | tail -n 1 > $P/bench_under_trace.json
echo done
