#!/bin/bash
# round 4 (final code): the base prefetch modes of the 29-bit accumulation again (set_variant 0 / bit 13 / bit 17)
mkdir -p gpurun_out
timeout -k 10 600 python tools/tune_msm.py --log-n 24 26 --variants 0 8192 131072 --rounds 2 > gpurun_out/ab_prefetch_r04.log 2>&1
