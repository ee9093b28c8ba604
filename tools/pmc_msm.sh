#!/bin/bash
# PMC counters of the MSM kernels (one counter group per rocprofv3 pass):
#   tools/pmc_msm.sh <tag> [tune_msm args]   (TACHYON_MI355X_LIB selects a build)
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
ARGS=${*:-"--log-n 26 --c 20 --reps 1"}
i=0
for grp in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES" \
           "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INST_LEVEL_VMEM" \
           "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F32"; do
  i=$((i+1))
  rc=0
  timeout -k 10 300 rocprofv3 --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 tools/tune_msm.py $ARGS > $OUT/p$i.log 2>&1 || rc=$?
  echo "pass $i rc=$rc"
  # a timeout, abort or crash ends the script (no further GPU work); rc 1 = counter rejected
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
echo done
