#!/bin/bash
# msum v7 (4x4 register tiles) + split-K in two subtrees (A/B).  Kernel/batch tests, benches, v7 profile.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread > gpurun_out/p29_k.log 2>&1 || { tail -30 gpurun_out/p29_k.log; exit 1; }
tail -1 gpurun_out/p29_k.log
for v in RWKV_MI355X_QG_SPLIT2=0 RWKV_MI355X_QG_SPLIT2=1; do
  env $v timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --skip-cpu --seq-reps 0 --abi-steps 0 --batch 32,64,128 > gpurun_out/p29.log 2>&1 || { tail -5 gpurun_out/p29.log; exit 1; }
  grep -E "batched" gpurun_out/p29.log | sed "s/^/[$v] /"
done
for c in v7-2b9-q5_1 v5-7b-q4_1; do
  timeout -k 10 400 python3 bench.py --config $c --steps 8 --warmup 2 --batch "32" --seq-reps 2 --abi-steps 0 --skip-cpu --timing-steps 1 > gpurun_out/p29_$c.log 2>&1 || { tail -5 gpurun_out/p29_$c.log; exit 1; }
  grep -E "seq-eval|batched" gpurun_out/p29_$c.log | sed "s/^/[$c] /" | cut -c1-160
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_v7seq11 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config v7-2b9-q5_1 --steps 2 --warmup 1 --batch "" --seq-reps 2 --abi-steps 0 --skip-cpu --timing-steps 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_v7seq11.log 2>&1 || exit 1
python3 $GRAFT_REPO_ROOT/tools/top_kernels.py $GRAFT_REPO_ROOT/gpurun_out/prof_v7seq11/run_kernel_stats.csv 8
echo done
