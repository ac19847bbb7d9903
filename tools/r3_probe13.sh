#!/bin/bash
# fmm (unconditional ring) + f32-MFMA mix5: kernel and parity tests, then batched / seq bench A/B.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
true

timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/p13_p.log 2>&1 || { tail -30 gpurun_out/p13_p.log; exit 1; }
tail -1 gpurun_out/p13_p.log
for v in "RWKV_MI355X_FMM=0 RWKV_MI355X_MIX5_MFMA=0" X=1; do
  env $v timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --skip-cpu --seq-reps 2 --abi-steps 0 --batch 32,64,128 > gpurun_out/p13.log 2>&1 || { tail -5 gpurun_out/p13.log; exit 1; }
  grep -E "batched|seq-eval" gpurun_out/p13.log | sed "s/^/[$v] /"
done
echo done
