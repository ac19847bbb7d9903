#!/bin/bash
# rocprofv3 kernel summary of the batched decode (B contexts per step) -- tools/, run on the GPU box
B=${1:-8}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_batch$B -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 --batch $B --batch-steps 20 --seq-reps 0 --abi-steps 0 \
  --skip-cpu --timing-steps 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_batch$B.log 2>&1
