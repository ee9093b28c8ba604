#!/bin/bash
# round 4 (final code): batched vs separate MSMs, then the rocprofv3 evidence (trace + PMC passes)
mkdir -p gpurun_out
timeout -k 10 300 python tools/batch_probe.py --log-len 10 12 14 16 --count 8 32 > gpurun_out/batch_probe.log 2>&1 &&
bash tools/profile_round.sh r04c > gpurun_out/profile_r04c.log 2>&1
