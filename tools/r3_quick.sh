#!/bin/bash
# Quick GPU cycle: the GPU test suite, a decode-only bench line and the decode phase stamps.
# Usage: tools/r3_quick.sh TAG [notests]
TAG=${1:-q}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
if [ "$2" != notests ]; then
  timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
  tail -2 gpurun_out/${TAG}_gputest.log
fi
timeout -k 10 300 python3 bench.py --steps 256 --skip-cpu --seq-reps 2 --batch "" --abi-steps 32 > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
grep -E "decode:|seq-eval|ABI" gpurun_out/${TAG}_bench.log
if [ -f rwkv.cppy_amd/build_stamp/librwkv.so ]; then
  timeout -k 10 200 python3 tools/stamp_run.py v6-1b6-q4_0 > gpurun_out/${TAG}_stamps.txt 2>&1 || { tail -5 gpurun_out/${TAG}_stamps.txt; exit 1; }
  sed -n 1,10p gpurun_out/${TAG}_stamps.txt
fi
echo done
