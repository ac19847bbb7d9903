cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -q -p no:cacheprovider --timeout 200 --timeout-method thread -x -k "decode or fixtures or timing or device_resident" > gpurun_out/gpu_r2j.log 2>&1
echo EXIT $? >> gpurun_out/gpu_r2j.log
for cfg in "0 64" "1 64" "1 128" "0 64" "1 32" "1 256"; do
  set -- $cfg
  RWKV_MI355X_PREFETCH=$1 RWKV_MI355X_PREFETCH_BLOCKS=$2 timeout -k 10 200 python bench.py --steps 128 --warmup 16 --skip-cpu --seq-reps 0 --abi-steps 0 > gpurun_out/bench_r2j_$1_$2.json 2> gpurun_out/bench_r2j_$1_$2_$RANDOM.err || exit 1
done
