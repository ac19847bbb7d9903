#!/bin/bash
# LDS-staged k_fmm: kernel tests, batched decode A/B (FMM on/off), rocprof of the B=128 step.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "matmul_kernel" > gpurun_out/p14_k.log 2>&1 || { tail -30 gpurun_out/p14_k.log; exit 1; }
tail -1 gpurun_out/p14_k.log
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread > gpurun_out/p14_b.log 2>&1 || { tail -30 gpurun_out/p14_b.log; exit 1; }
tail -1 gpurun_out/p14_b.log
for v in RWKV_MI355X_FMM=0 RWKV_MI355X_FMM=1; do
  env $v timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --skip-cpu --seq-reps 0 --abi-steps 0 --batch 16,32,64,128 > gpurun_out/p14.log 2>&1 || { tail -5 gpurun_out/p14.log; exit 1; }
  grep -E "batched" gpurun_out/p14.log | sed "s/^/[$v] /"
done
bash tools/batch_prof.sh 128 || exit 1
python3 tools/top_kernels.py gpurun_out/prof_batch128/run_kernel_stats.csv 12
echo done
