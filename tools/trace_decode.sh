#!/bin/bash
# rocprofv3 kernel trace of a few decode tokens (no timing pass) -- tools/, on the GPU box
TAG=${1:-dec}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/tr_$TAG -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 8 --warmup 2 --batch "" --seq-reps 0 --abi-steps 0 --skip-cpu --timing-steps 1 \
  > $GRAFT_REPO_ROOT/gpurun_out/tr_$TAG.log 2>&1
