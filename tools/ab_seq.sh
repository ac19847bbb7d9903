#!/bin/bash
# A/B of sequence-eval variants (env switches) on the bench workload -- tools/, on the GPU box.
# Usage: tools/ab_seq.sh "VAR=a" "VAR=b" ...   (BATCH env: batched-decode sizes, default none;
# CFG env: bench config, default v6-1b6-q4_0)
cd $GRAFT_REPO_ROOT
for v in "$@"; do
  env $v timeout -k 10 300 python3 bench.py --config ${CFG:-v6-1b6-q4_0} --steps 8 --warmup 2 --skip-cpu --seq-reps 5 \
    --abi-steps 0 --batch "${BATCH:-}" --timing-steps 1 --pipe-stages 0 2>&1 | grep -E "seq-eval|seq GEMM|batched|Error|error" | sed "s/^/[$v] /"
done
