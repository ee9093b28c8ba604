#!/bin/bash
# The one GPU-box runner (it replaces the per-round tools/gpu_r0*.sh drivers;
# their recipes are in git history and in each profiles/<tag>/ README):
#
#   tools/gpu_run.sh TAG STEP [STEP ...]
#
# STEP is one of
#   smoke              python __graft_entry__.py smoke
#   tests=ARGS         python -u -m pytest -m gpu -x -v --timeout 300 ARGS   (ARGS default: tests;
#                      evaluated by the shell: quote a -k expression inside it)
#   bench=ARGS         python bench.py ARGS; the JSON line -> gpurun_out/TAG/bench_<k>.json
#   profile=ARGS       tools/profile_round.sh TAG ARGS (trace + PMC passes of a bench command)
#   pmc=COUNTERS@ARGS  one rocprofv3 --pmc pass over python bench.py ARGS (counters space-separated)
#   cmd=COMMAND        any other command (A/B probes: python tools/... )
#
# Each step runs under its own time limit (STEP_TIMEOUT seconds, default 900)
# and writes its log to gpurun_out/TAG/<k>_<kind>.log.  A fault, abort,
# crash or timeout (rc other than 0 and 1) ends the script at that step: no
# further GPU work runs in the call.  rc 1 (test or check failures) goes on.
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
LIMIT=${STEP_TIMEOUT:-900}
worst=0
k=0
for step in "$@"; do
  k=$((k + 1))
  kind=${step%%=*}
  arg=""
  [ "$kind" != "$step" ] && arg=${step#*=}
  log=$OUT/${k}_${kind}.log
  echo "[$(date +%T)] step $k: $step" | tee -a "$OUT/steps.log"
  case $kind in
    smoke) timeout -k 10 "$LIMIT" python __graft_entry__.py smoke > "$log" 2>&1 ;;
    tests) eval "timeout -k 10 $LIMIT python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread \
             ${arg:-tests}" > "$log" 2>&1 ;;
    bench) eval "timeout -k 10 $LIMIT python bench.py $arg" > "$log" 2>&1 ;;
    profile) timeout -k 10 "$LIMIT" bash tools/profile_round.sh "$TAG" $arg > "$log" 2>&1 ;;
    pmc) counters=${arg%%@*}
         bargs=${arg#*@}
         timeout -s KILL 300 rocprofv3 --pmc $counters -d "$OUT/pmc_$k" -o run --output-format csv -- \
           python3 bench.py $bargs > "$log" 2>&1 ;;
    cmd) timeout -k 10 "$LIMIT" bash -c "$arg" > "$log" 2>&1 ;;
    *) echo "unknown step $step" | tee -a "$OUT/steps.log"; exit 2 ;;
  esac
  rc=$?
  echo "[$(date +%T)] step $k rc=$rc" | tee -a "$OUT/steps.log"
  tail -n 3 "$log"
  if [ "$kind" = bench ] && [ $rc -eq 0 ]; then
    grep '^{"metric"' "$log" | tail -n 1 > "$OUT/bench_$k.json"
  fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping: step $k ended with rc=$rc" | tee -a "$OUT/steps.log"
    exit $rc
  fi
  [ $rc -gt $worst ] && worst=$rc
done
exit $worst
