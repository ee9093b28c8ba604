set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_full_size.py tests/test_gpu_multi_device.py tests/test_gpu_harness.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_msm.log 2>&1 || exit 1
LIB_A=ab/lib_base.so LIB_B=tachyon_amd/libtachyon_mi355x.so timeout -k 10 400 tools/ab_libs.sh 3 --log-n 16 18 20 22 --reps 5 || exit 2
LIB_A=ab/lib_base.so LIB_B=tachyon_amd/libtachyon_mi355x.so timeout -k 10 300 tools/ab_libs.sh 2 --log-n 26 --reps 3 || exit 3
