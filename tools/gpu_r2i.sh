cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -q -p no:cacheprovider --timeout 200 --timeout-method thread -x -k "decode or fixtures or quantized" > gpurun_out/gpu_r2i.log 2>&1
echo EXIT $? >> gpurun_out/gpu_r2i.log
for cfg in "2 64" "4 64" "8 64" "4 256"; do
  set -- $cfg
  RWKV_MI355X_MVA_R=$1 RWKV_MI355X_MAA_CPW=$2 timeout -k 10 200 python bench.py --steps 128 --warmup 16 --skip-cpu --seq-reps 0 --abi-steps 0 > gpurun_out/bench_r2i_$1_$2.json 2> gpurun_out/bench_r2i_$1_$2.err || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r2i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 64 --skip-cpu --seq-reps 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_r2i.log 2>&1
