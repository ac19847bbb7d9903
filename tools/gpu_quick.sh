#!/bin/bash
# Quick GPU cycle on the box: parity tests, then a rocprofv3 kernel trace of a short bench run.
# Usage: tools/gpu_quick.sh TAG [skip-tests]
TAG=${1:-x}
cd $GRAFT_REPO_ROOT
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -x > gpurun_out/gpu_$TAG.log 2>&1
  rc=$?
  echo EXIT $rc >> gpurun_out/gpu_$TAG.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 64 --skip-cpu --seq-reps 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
