#!/bin/bash
# A/B of batched-decode variants (env switches) -- tools/, on the GPU box
cd $GRAFT_REPO_ROOT
for v in "$@"; do
  env $v timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --skip-cpu --seq-reps 0 --abi-steps 0 --batch 16,32,64,128 --timing-steps 1 2>&1 | grep -E "batched decode" | sed "s/^/[$v] /"
done
