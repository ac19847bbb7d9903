#!/bin/bash
# k_fmm: zero-class tail as aligned +0 nodes.  Kernel tests + fmm probe + v7 bench.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread > gpurun_out/p34_k.log 2>&1 || { tail -30 gpurun_out/p34_k.log; exit 1; }
tail -1 gpurun_out/p34_k.log
timeout -k 10 120 tools/pbin/fmm_probe > gpurun_out/p34_fmm.txt 2>&1 || { cat gpurun_out/p34_fmm.txt; exit 1; }
cat gpurun_out/p34_fmm.txt
timeout -k 10 400 python3 bench.py --config v7-2b9-q5_1 --steps 8 --warmup 2 --batch "32" --seq-reps 2 --abi-steps 0 --skip-cpu --timing-steps 1 > gpurun_out/p34_v7.log 2>&1 || { tail -5 gpurun_out/p34_v7.log; exit 1; }
grep -E "seq-eval|batched" gpurun_out/p34_v7.log | cut -c1-160
echo done
