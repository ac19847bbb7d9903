#!/bin/bash
# A/B of decode/sequence variants (env switches) on one BASELINE configuration -- tools/, on the GPU box.
# Usage: tools/ab_cfg.sh CONFIG "ENV=1" "ENV=0" ...
cd $GRAFT_REPO_ROOT
CFG=$1; shift
for v in "$@"; do
  env $v timeout -k 10 300 python3 bench.py --config $CFG --steps 128 --warmup 8 --skip-cpu --seq-reps 2 --abi-steps 0 --batch "" 2>&1 | grep -E "decode:|seq-eval" | sed "s/^/[$v] /" || exit 1
done
