#!/bin/bash
# k_fmm A/B on the batched decode and its kernel time.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in RWKV_MI355X_FMM=0 RWKV_MI355X_FMM=1; do
  env $v timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --skip-cpu --seq-reps 0 --abi-steps 0 --batch 32,64,128 > gpurun_out/p12.log 2>&1 || { tail -5 gpurun_out/p12.log; exit 1; }
  grep -E "batched" gpurun_out/p12.log | sed "s/^/[$v] /"
done
bash tools/batch_prof.sh 128 || exit 1
python3 tools/top_kernels.py gpurun_out/prof_batch128/run_kernel_stats.csv 12
echo done
