#!/bin/bash
# NTT pass-kernel A/B under rocprofv3 (GPU box): probe timings, kernel trace,
# and PMC passes (one counter group per run).  tools/ntt_pmc.sh <tag> [probe args]
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/ntt_$TAG
mkdir -p $OUT
ARGS=${*:-"--log-n 24 --reps 10 --rounds 2"}
timeout -k 10 120 python3 tools/ntt_probe.py $ARGS > $OUT/probe.log 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/ntt_probe.py --rounds 1 --reps 3 > $OUT/trace.log 2>&1 || exit $?
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  rc=0
  timeout -k 10 120 rocprofv3 --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 tools/ntt_probe.py --rounds 1 --reps 2 > $OUT/p$i.log 2>&1 || rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
echo done
