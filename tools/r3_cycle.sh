#!/bin/bash
# Round-3 measurement cycle on the GPU box: GPU tests, smoke, the default bench line and the
# rocprofv3 kernel-trace stats of the bench workload.  Every GPU step has its own time limit;
# the script stops at the first failure.  Usage: tools/r3_cycle.sh TAG [tests|notests]
TAG=${1:-r3}
MODE=${2:-tests}
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out
if [ "$MODE" = tests ]; then
  timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
  tail -3 gpurun_out/${TAG}_gputest.log
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { cat gpurun_out/${TAG}_smoke.log; exit 1; }
  tail -1 gpurun_out/${TAG}_smoke.log
fi
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -15 gpurun_out/${TAG}_bench.log; exit 1; }
grep '^{' gpurun_out/${TAG}_bench.log > gpurun_out/${TAG}_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof_${TAG} -o run --output-format csv -- \
  python3 $ROOT/bench.py --steps 64 --skip-cpu --seq-reps 1 --batch 8 --abi-steps 4 > $ROOT/gpurun_out/prof_${TAG}.log 2>&1 || { tail -5 $ROOT/gpurun_out/prof_${TAG}.log; exit 1; }
echo done
