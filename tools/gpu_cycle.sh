#!/bin/bash
# One GPU cycle on the box: parity tests, bench (with the CPU baseline), rocprofv3 kernel trace.
# Usage: tools/gpu_cycle.sh TAG [skip-tests]
TAG=${1:-x}
cd $GRAFT_REPO_ROOT
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -x > gpurun_out/gpu_$TAG.log 2>&1
  rc=$?
  echo EXIT $rc >> gpurun_out/gpu_$TAG.log
  # test failures (1) still allow a measurement; a fault, abort or timeout ends the call
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 64 --skip-cpu --seq-reps 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
