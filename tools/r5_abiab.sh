#!/bin/bash
# ABI decode rate A/B over env knobs: tools/r5_abiab.sh "VAR=a VAR2=b" ...
cd $GRAFT_REPO_ROOT
for v in "$@"; do
  for k in pageable pinned; do
    env $v timeout -k 10 120 python3 tools/abi_trace.py $k 96 2>/dev/null | sed "s/^/[$v] /" || exit 1
  done
done
