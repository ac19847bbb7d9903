#!/bin/bash
# Round-2 GPU cycle on the box: parity tests, arithmetic probe, the driver's bench command, and a
# rocprofv3 kernel-trace of a short bench.  Every GPU step has its own time limit; a fault, abort
# or timeout ends the call.   Usage: tools/r2_cycle.sh TAG [skip-tests] [skip-prof]
TAG=${1:-x}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -x > gpurun_out/gpu_$TAG.log 2>&1
  rc=$?
  echo EXIT $rc >> gpurun_out/gpu_$TAG.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ -x tools/bin/arith_probe ] && [ ! -f gpurun_out/arith_probe.bin ]; then
  timeout -k 10 60 tools/bin/arith_probe gpurun_out/arith_probe.bin > gpurun_out/arith_$TAG.log 2>&1 || exit 2
fi
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 3
if [ "$3" != "skip-prof" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 64 --skip-cpu --seq-reps 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
fi
