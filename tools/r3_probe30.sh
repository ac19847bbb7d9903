#!/bin/bash
# msum: tile form (<= 4 blocks per class) + row form (5-8).  Tests + _1 benches.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_batch.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/p30_k.log 2>&1 || { tail -30 gpurun_out/p30_k.log; exit 1; }
tail -1 gpurun_out/p30_k.log
for c in v7-2b9-q5_1 v5-7b-q4_1; do
  timeout -k 10 400 python3 bench.py --config $c --steps 8 --warmup 2 --batch "32" --seq-reps 2 --abi-steps 0 --skip-cpu --timing-steps 1 > gpurun_out/p30_$c.log 2>&1 || { tail -5 gpurun_out/p30_$c.log; exit 1; }
  grep -E "seq-eval|batched" gpurun_out/p30_$c.log | sed "s/^/[$c] /" | cut -c1-160
done
echo done
