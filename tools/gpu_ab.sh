#!/bin/bash
# GPU cycle used while tuning: parity tests, a short bench line, and a rocprofv3 kernel-trace of
# the sequence eval + single decode (no batched decode).  Every GPU step has its own time limit and
# the first failure ends the call.   Usage: tools/gpu_ab.sh TAG [skip-tests] [skip-prof]
TAG=${1:-x}
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_$TAG.log 2>&1
  rc=$?
  tail -3 gpurun_out/gpu_$TAG.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/gpu_$TAG.log | head -30; exit $rc; fi
fi
timeout -k 10 300 python bench.py --steps 64 --warmup 8 --skip-cpu --seq-reps 3 --abi-steps 4 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 4; }
grep -E "decode:|seq-eval|k_mv |seq GEMM|batch" gpurun_out/bench_$TAG.err
if [ "$3" != "skip-prof" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof_$TAG -o run --output-format csv -- \
    python3 $ROOT/bench.py --steps 32 --skip-cpu --seq-reps 2 --batch "" --abi-steps 0 > $ROOT/gpurun_out/prof_$TAG.log 2>&1 || exit 5
  python3 $ROOT/tools/top_kernels.py $ROOT/gpurun_out/prof_$TAG/run_kernel_stats.csv
fi
echo done
