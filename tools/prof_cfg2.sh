#!/bin/bash
# rocprofv3 kernel stats of one BASELINE configuration's bench (decode + sequence eval).
# Usage: tools/prof_cfg2.sh CONFIG TAG
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof_$2 -o run --output-format csv -- \
  python3 $ROOT/bench.py --config $1 --steps 32 --skip-cpu --seq-reps 2 --batch "" --abi-steps 0 > $ROOT/gpurun_out/prof_$2.log 2>&1 || { tail -5 $ROOT/gpurun_out/prof_$2.log; exit 5; }
grep -E "decode:|seq-eval" $ROOT/gpurun_out/prof_$2.log
python3 $ROOT/tools/top_kernels.py $ROOT/gpurun_out/prof_$2/run_kernel_stats.csv 26
