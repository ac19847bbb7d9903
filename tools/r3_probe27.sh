#!/bin/bash
# wkv7 token loop with the next token's LDS operands read ahead: v7 parity + bench.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread > gpurun_out/p27_t.log 2>&1 || { tail -30 gpurun_out/p27_t.log; exit 1; }
tail -1 gpurun_out/p27_t.log
timeout -k 10 400 python3 bench.py --config v7-2b9-q5_1 --steps 8 --warmup 2 --batch "32" --seq-reps 2 --abi-steps 0 --skip-cpu --timing-steps 1 > gpurun_out/p27_v7.log 2>&1 || { tail -5 gpurun_out/p27_v7.log; exit 1; }
grep -E "seq-eval|decode" gpurun_out/p27_v7.log | cut -c1-160
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_v7seq10 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config v7-2b9-q5_1 --steps 2 --warmup 1 --batch "" --seq-reps 2 --abi-steps 0 --skip-cpu --timing-steps 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_v7seq10.log 2>&1 || exit 1
python3 $GRAFT_REPO_ROOT/tools/top_kernels.py $GRAFT_REPO_ROOT/gpurun_out/prof_v7seq10/run_kernel_stats.csv 8
echo done
