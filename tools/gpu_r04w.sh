#!/bin/bash
# round 4 (final library): rocprofv3 trace + PMC passes of the bench command
mkdir -p gpurun_out
bash tools/profile_round.sh r04d > gpurun_out/profile_r04d.log 2>&1
