#!/bin/bash
# A/B environment settings on one library (alternating):
#   tools/ab_env.sh <rounds> <tool.py> "<ENV_A>" "<ENV_B>" [...] -- <tool args>  -> gpurun_out/ab_env.log
set -o pipefail
mkdir -p gpurun_out
R=$1; TOOL=$2; shift 2
envs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
shift || true
for i in $(seq 1 $R); do
  for e in "${envs[@]}"; do
    echo "== $e" >> gpurun_out/ab_env.log
    env $e timeout -k 10 180 python $TOOL "$@" >> gpurun_out/ab_env.log 2>&1 || exit $?
  done
done
