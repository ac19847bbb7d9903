cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/gpu_r2h.log 2>&1
echo EXIT $? >> gpurun_out/gpu_r2h.log
timeout -k 10 120 tools/bin/mv_probe > gpurun_out/mvprobe_r2h.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 64 --warmup 8 --skip-cpu --seq-reps 2 > gpurun_out/bench_r2h.json 2> gpurun_out/bench_r2h.err
