mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_concurrency.py tests/test_gpu_configs.py tests/test_gpu_parity.py > gpurun_out/r6_ffe_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r6_ffe_tests.txt; [ $rc = 0 ] || exit $rc
tools/ab_lib.sh v4-169m-q8_0 3 early=this late=rwkv.cppy_amd/build_late/librwkv.so > gpurun_out/r6_ab_ffco_early.txt 2>&1 || exit 1
cat gpurun_out/r6_ab_ffco_early.txt
