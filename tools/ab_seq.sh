#!/bin/bash
# A/B of sequence-eval variants (env switches) on the bench workload -- tools/, on the GPU box
cd $GRAFT_REPO_ROOT
for v in "$@"; do
  env $v timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --skip-cpu --seq-reps 5 --abi-steps 0 --batch "" --timing-steps 1 2>&1 | grep -E "seq-eval|seq GEMM" | sed "s/^/[$v] /"
done
