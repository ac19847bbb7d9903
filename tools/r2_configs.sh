#!/bin/bash
# Round-2 bench lines of the other BASELINE configs (tools/, on the GPU box); each step bounded,
# stop at the first failure.
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
for CFG in ${CFGS:-v7-2b9-q5_1 v4-169m-q8_0 v5-7b-q4_1}; do
  timeout -k 10 500 python3 -u bench.py --config $CFG --skip-cpu --batch 8,64 > gpurun_out/r2_cfg_$CFG.log 2>&1 \
    || { tail -5 gpurun_out/r2_cfg_$CFG.log; exit 1; }
  grep '^{' gpurun_out/r2_cfg_$CFG.log > gpurun_out/r2_cfg_$CFG.json
  echo "$CFG done"
done
