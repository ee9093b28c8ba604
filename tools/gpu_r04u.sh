#!/bin/bash
# round 4 (final library): the whole GPU suite and smoke()
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_final.log 2>&1 &&
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke_final.log 2>&1
