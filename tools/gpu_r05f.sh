#!/bin/bash
# round 5: profile + default bench line of the final library
bash tools/profile_round.sh r05f || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_full_r05f.log 2>&1
