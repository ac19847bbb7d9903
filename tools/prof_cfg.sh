#!/bin/bash
# rocprofv3 kernel stats of one BASELINE config's bench workload -- tools/, on the GPU box
CFG=${1:-v7-2b9-q5_1}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$CFG -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/bench.py --config $CFG --steps 16 --warmup 4 --skip-cpu --seq-reps 1 --abi-steps 0 --batch "" \
  --timing-steps 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_$CFG.log 2>&1
