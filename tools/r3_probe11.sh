#!/bin/bash
# f32-MFMA (pipelined) + batch GEMM threshold 16: kernel tests, batch tests, full suite, bench, v7 bench.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/p11_k.log 2>&1 || { tail -30 gpurun_out/p11_k.log; exit 1; }
tail -1 gpurun_out/p11_k.log
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_batch.py -x -q --timeout 120 --timeout-method thread > gpurun_out/p11_b.log 2>&1 || { tail -30 gpurun_out/p11_b.log; exit 1; }
tail -1 gpurun_out/p11_b.log
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/p11_gputest.log 2>&1 || { tail -30 gpurun_out/p11_gputest.log; exit 1; }
tail -1 gpurun_out/p11_gputest.log
timeout -k 10 300 python3 bench.py --steps 64 --skip-cpu --seq-reps 2 --abi-steps 0 --batch 8,16,32,64,128 > gpurun_out/p11_bench.log 2>&1 || { tail -5 gpurun_out/p11_bench.log; exit 1; }
grep -E "decode|seq-eval" gpurun_out/p11_bench.log
timeout -k 10 400 python3 bench.py --config v7-2b9-q5_1 --steps 8 --warmup 2 --batch "" --seq-reps 2 --abi-steps 0 --skip-cpu --timing-steps 1 > gpurun_out/p11_v7.log 2>&1 || { tail -5 gpurun_out/p11_v7.log; exit 1; }
grep -E "seq-eval|decode:" gpurun_out/p11_v7.log
echo done
