mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py -k "wide" > gpurun_out/r6_wide_tests.txt 2>&1
rc=$?; tail -5 gpurun_out/r6_wide_tests.txt; exit $rc
