#!/bin/bash
# Round-2 measurement on the GPU box (tools/): GPU tests, smoke, the default bench line, the
# rocprofv3 kernel-trace stats of the bench workload.  Every step bounded; stop at the first failure.
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_gputest.log 2>&1 || { tail -20 gpurun_out/r2_gputest.log; exit 1; }
tail -2 gpurun_out/r2_gputest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_smoke.log 2>&1 || { cat gpurun_out/r2_smoke.log; exit 1; }
tail -1 gpurun_out/r2_smoke.log
timeout -k 10 400 python3 bench.py > gpurun_out/r2_bench.log 2>&1 || { tail -5 gpurun_out/r2_bench.log; exit 1; }
grep '^{' gpurun_out/r2_bench.log > gpurun_out/r2_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof_r2 -o run --output-format csv -- \
  python3 $ROOT/bench.py --steps 64 --skip-cpu --seq-reps 1 --batch 8 --abi-steps 4 > $ROOT/gpurun_out/prof_r2.log 2>&1 || exit 1
echo done
