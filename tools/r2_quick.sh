#!/bin/bash
# Quick GPU cycle: parity tests, stamped decode token, short bench.  Usage: tools/r2_quick.sh TAG [skip-tests]
TAG=${1:-x}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_$TAG.log 2>&1
  rc=$?
  tail -3 gpurun_out/gpu_$TAG.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/gpu_$TAG.log | head -20; exit $rc; fi
fi
if [ -f rwkv.cppy_amd/build_stamp/librwkv.so ]; then
  timeout -k 10 120 python tools/stamp_run.py > gpurun_out/stamp_$TAG.txt 2>&1 || exit 3
  tail -8 gpurun_out/stamp_$TAG.txt
fi
timeout -k 10 300 python bench.py --steps 64 --warmup 8 --skip-cpu --seq-reps 2 --abi-steps 4 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 4
grep -E "decode:|seq-eval|k_mv |seq GEMM" gpurun_out/bench_$TAG.err
