#!/bin/bash
# batched decode after split-K + f32 MFMA: kernel summaries at B = 64 / 128, the GEMM-route
# threshold at B = 16 / 24 / 32, and the v7 sequence eval (F16 LoRA now on the f32 MFMA).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for B in 64 128; do bash tools/batch_prof.sh $B || exit 1; grep -E "batched" gpurun_out/prof_batch$B.log; done
for m in 16 24 32 48; do
  RWKV_MI355X_BATCH_GEMM_MIN=$m timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --skip-cpu --seq-reps 0 --abi-steps 0 --batch 16,24,32,48 > gpurun_out/p10_gm.log 2>&1 || { tail -5 gpurun_out/p10_gm.log; exit 1; }
  grep -E "batched" gpurun_out/p10_gm.log | sed "s/^/[min $m] /"
done
timeout -k 10 400 python3 bench.py --config v7-2b9-q5_1 --steps 8 --warmup 2 --batch "" --seq-reps 2 --abi-steps 0 --skip-cpu --timing-steps 1 > gpurun_out/p10_v7.log 2>&1 || { tail -5 gpurun_out/p10_v7.log; exit 1; }
grep -E "seq-eval|decode:" gpurun_out/p10_v7.log
echo done
