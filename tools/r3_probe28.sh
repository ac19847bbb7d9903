#!/bin/bash
# split-K in two subtrees (A/B behind RWKV_MI355X_QG_SPLIT2) on the batched decode.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "split" > gpurun_out/p28_k.log 2>&1 || { tail -30 gpurun_out/p28_k.log; exit 1; }
tail -1 gpurun_out/p28_k.log
for v in RWKV_MI355X_QG_SPLIT2=0 RWKV_MI355X_QG_SPLIT2=1; do
  env $v timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --skip-cpu --seq-reps 0 --abi-steps 0 --batch 32,64,128 > gpurun_out/p28.log 2>&1 || { tail -5 gpurun_out/p28.log; exit 1; }
  grep -E "batched" gpurun_out/p28.log | sed "s/^/[$v] /"
done
echo done
