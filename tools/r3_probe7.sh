#!/bin/bash
# Kernel summaries of the batched decode at B = 32, 64 and 128 and of the v7-2.9B sequence eval.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for B in 32 64 128; do
  bash tools/batch_prof.sh $B || exit 1
  grep -E "batched" gpurun_out/prof_batch$B.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_v7seq -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/bench.py --config v7-2b9-q5_1 --steps 8 --warmup 2 --batch "" --seq-reps 2 --abi-steps 0 --skip-cpu --timing-steps 1 \
  > $GRAFT_REPO_ROOT/gpurun_out/prof_v7seq.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/prof_v7seq.log; exit 1; }
grep -E "seq-eval|decode:" $GRAFT_REPO_ROOT/gpurun_out/prof_v7seq.log
echo done
