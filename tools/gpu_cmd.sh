mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_concurrency.py tests/test_gpu_configs.py tests/test_gpu_parity.py > gpurun_out/r6_ffco_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r6_ffco_tests.txt; [ $rc = 0 ] || exit $rc
tools/ab_lib.sh v6-1b6-q4_0 3 ffco=this off=this@RWKV_MI355X_DECODE_FUSION=63 > gpurun_out/r6_ab_ffco_v6.txt 2>&1 || exit 1
cat gpurun_out/r6_ab_ffco_v6.txt
tools/ab_lib.sh v4-169m-q8_0 2 ffco=this off=this@RWKV_MI355X_DECODE_FUSION=63 > gpurun_out/r6_ab_ffco_v4.txt 2>&1 || exit 1
cat gpurun_out/r6_ab_ffco_v4.txt
