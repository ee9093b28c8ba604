#!/bin/bash
# Kernel timelines of the small MSMs (launch gaps, the chain read-back, the
# serial reduction levels):  ./tools/trace_small.sh <tag> [log_n ...]
set -e
TAG=${1:-small}
shift || true
SIZES=${@:-16 20}
export TMPDIR=/tmp
OUT=gpurun_out/trace_$TAG
mkdir -p $OUT
for lg in $SIZES; do
  timeout -k 10 180 rocprofv3 --kernel-trace -d $OUT/t$lg -o run --output-format csv -- \
    python tools/tune_msm.py --log-n $lg --reps 3 > $OUT/tune_$lg.log 2>&1
  python tools/timeline.py $(find $OUT/t$lg -name run_kernel_trace.csv) \
    > $OUT/timeline_$lg.txt
done
echo done
