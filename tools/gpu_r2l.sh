cd $GRAFT_REPO_ROOT
for v in 0 1 0 1; do
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python bench.py --steps 128 --warmup 16 --skip-cpu --seq-reps 2 --abi-steps 0 > gpurun_out/bench_r2l_$v.json 2> gpurun_out/bench_r2l_${v}_$RANDOM.err || exit 1
done
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 120 tools/bin/mv_probe > gpurun_out/mvprobe_r2l.log 2>&1
