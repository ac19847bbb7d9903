mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_concurrency.py tests/test_gpu_configs.py tests/test_gpu_parity.py > gpurun_out/r6_coq8_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r6_coq8_tests.txt; [ $rc = 0 ] || exit $rc
tools/ab_lib.sh v6-1b6-q4_0 3 base=rwkv.cppy_amd/build_base/librwkv.so q8y=this kdev1=this@HIP_FORCE_DEV_KERNARG=1 kdev0=this@HIP_FORCE_DEV_KERNARG=0 > gpurun_out/r6_ab_coq8.txt 2>&1 || exit 1
cat gpurun_out/r6_ab_coq8.txt
for i in 1 2; do
  timeout -k 10 300 python tools/ab_seq.py --config v7-2b9-q5_1 --reps 3 --lib rwkv.cppy_amd/build_base/librwkv.so 2>&1 | tail -1 | sed 's/^/[base] /' || exit 1
  timeout -k 10 300 python tools/ab_seq.py --config v7-2b9-q5_1 --reps 3 2>&1 | tail -1 | sed 's/^/[this] /' || exit 1
done > gpurun_out/r6_ab_wkv7.txt
cat gpurun_out/r6_ab_wkv7.txt
