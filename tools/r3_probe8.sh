#!/bin/bash
# f32-MFMA numerics probe, the GPU test suite (split-K GEMM included) and the batched-decode bench.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 60 tools/pbin/mfma_f32_probe > gpurun_out/p8_mfma.txt 2>&1 || { cat gpurun_out/p8_mfma.txt; exit 1; }
cat gpurun_out/p8_mfma.txt
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/p8_gputest.log 2>&1 || { tail -30 gpurun_out/p8_gputest.log; exit 1; }
tail -2 gpurun_out/p8_gputest.log
timeout -k 10 300 python3 bench.py --steps 64 --skip-cpu --seq-reps 2 --abi-steps 0 > gpurun_out/p8_bench.log 2>&1 || { tail -5 gpurun_out/p8_bench.log; exit 1; }
grep -E "decode|seq-eval" gpurun_out/p8_bench.log
echo done
