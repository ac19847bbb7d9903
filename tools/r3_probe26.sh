#!/bin/bash
# round-3b measurement: default bench + rocprof stats, batched B=128 profile, config benches.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/r3_cycle.sh r3b notests || exit 1
grep -E "decode|seq-eval" gpurun_out/r3b_bench.log | cut -c1-160
bash tools/batch_prof.sh 128 || exit 1
python3 tools/top_kernels.py gpurun_out/prof_batch128/run_kernel_stats.csv 16
for c in v4-169m-q8_0 v7-2b9-q5_1 v5-7b-q4_1; do
  timeout -k 10 400 python3 bench.py --config $c --steps 16 --warmup 4 --batch "8,64" --seq-reps 2 --abi-steps 0 --skip-cpu > gpurun_out/r3b_cfg_$c.log 2>&1 || { tail -5 gpurun_out/r3b_cfg_$c.log; exit 1; }
  grep '^{' gpurun_out/r3b_cfg_$c.log > gpurun_out/r3b_cfg_$c.json
  grep -E "decode|seq-eval" gpurun_out/r3b_cfg_$c.log | cut -c1-160
done
echo done
