#!/bin/bash
# fmm for every float matmul over 32+ tokens: full GPU suite, v6 bench, v7 bench + v7 sequence profile.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/p15_gputest.log 2>&1 || { tail -30 gpurun_out/p15_gputest.log; exit 1; }
tail -1 gpurun_out/p15_gputest.log
timeout -k 10 300 python3 bench.py --steps 64 --skip-cpu --seq-reps 2 --abi-steps 0 --batch 32,64,128 > gpurun_out/p15_bench.log 2>&1 || { tail -5 gpurun_out/p15_bench.log; exit 1; }
grep -E "decode|seq-eval" gpurun_out/p15_bench.log
timeout -k 10 400 python3 bench.py --config v7-2b9-q5_1 --steps 8 --warmup 2 --batch "" --seq-reps 2 --abi-steps 0 --skip-cpu --timing-steps 1 > gpurun_out/p15_v7.log 2>&1 || { tail -5 gpurun_out/p15_v7.log; exit 1; }
grep -E "seq-eval|decode:" gpurun_out/p15_v7.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_v7seq -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config v7-2b9-q5_1 --steps 2 --warmup 1 --batch "" --seq-reps 2 --abi-steps 0 --skip-cpu --timing-steps 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_v7seq.log 2>&1 || exit 1
python3 $GRAFT_REPO_ROOT/tools/top_kernels.py $GRAFT_REPO_ROOT/gpurun_out/prof_v7seq/run_kernel_stats.csv 16
echo done
