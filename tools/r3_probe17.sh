#!/bin/bash
# msum v2 (tokens on lanes, load ring), batched mix5 on MFMA, ln_mix grid: tests + benches + v7 profile.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread > gpurun_out/p17_k.log 2>&1 || { tail -30 gpurun_out/p17_k.log; exit 1; }
tail -1 gpurun_out/p17_k.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/p17_gputest.log 2>&1 || { tail -30 gpurun_out/p17_gputest.log; exit 1; }
tail -1 gpurun_out/p17_gputest.log
timeout -k 10 300 python3 bench.py --steps 32 --skip-cpu --seq-reps 2 --abi-steps 0 --batch 16,32,64,128 > gpurun_out/p17_bench.log 2>&1 || { tail -5 gpurun_out/p17_bench.log; exit 1; }
grep -E "decode|seq-eval" gpurun_out/p17_bench.log | cut -c1-200
timeout -k 10 400 python3 bench.py --config v7-2b9-q5_1 --steps 8 --warmup 2 --batch "32,128" --seq-reps 2 --abi-steps 0 --skip-cpu --timing-steps 1 > gpurun_out/p17_v7.log 2>&1 || { tail -5 gpurun_out/p17_v7.log; exit 1; }
grep -E "seq-eval|decode" gpurun_out/p17_v7.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_v7seq3 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config v7-2b9-q5_1 --steps 2 --warmup 1 --batch "" --seq-reps 2 --abi-steps 0 --skip-cpu --timing-steps 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_v7seq3.log 2>&1 || exit 1
python3 $GRAFT_REPO_ROOT/tools/top_kernels.py $GRAFT_REPO_ROOT/gpurun_out/prof_v7seq3/run_kernel_stats.csv 12
echo done
