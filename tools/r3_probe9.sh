#!/bin/bash
# split-K GEMM: the kernel self-tests first (single entries), then the batched-decode tests (groups),
# then the whole GPU suite and the bench.  Stops at the first failure.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/p9_k.log 2>&1 || { tail -30 gpurun_out/p9_k.log; exit 1; }
tail -1 gpurun_out/p9_k.log
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_batch.py -x -q --timeout 120 --timeout-method thread > gpurun_out/p9_b.log 2>&1 || { tail -30 gpurun_out/p9_b.log; exit 1; }
tail -1 gpurun_out/p9_b.log
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/p9_gputest.log 2>&1 || { tail -30 gpurun_out/p9_gputest.log; exit 1; }
tail -1 gpurun_out/p9_gputest.log
timeout -k 10 300 python3 bench.py --steps 64 --skip-cpu --seq-reps 2 --abi-steps 0 > gpurun_out/p9_bench.log 2>&1 || { tail -5 gpurun_out/p9_bench.log; exit 1; }
grep -E "decode|seq-eval" gpurun_out/p9_bench.log
echo done
