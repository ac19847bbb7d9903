#!/bin/bash
# A/B of the ABI-decode host-state variants (env switches) -- tools/, on the GPU box
cd $GRAFT_REPO_ROOT
for v in "$@"; do
  env $v timeout -k 10 200 python3 bench.py --steps 16 --skip-cpu --seq-reps 0 --batch "" --abi-steps 64 --timing-steps 1 2>&1 | grep -E "ABI" | sed "s/^/[$v] /"
done
