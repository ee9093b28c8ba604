mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ntt.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ntt_tests.log 2>&1
rc=$?; echo "ntt rc=$rc" >> gpurun_out/ntt_tests.log
[ $rc -ne 0 ] && exit $rc
PYTEST_ARGS="--timeout 300 --timeout-method thread" GPU_TEST_TIMEOUT=800 bash tools/gpu_check.sh || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_r04b.log 2>&1
