#!/bin/bash
# Quick GPU cycle (round 4): a focused test file first (fails fast), then the GPU suite, a
# decode-only bench line and the decode phase stamps.  Every GPU step has its own time limit and
# the script stops at the first failure.
# Usage: tools/r4_quick.sh TAG [focus-pytest-args|-] [notests|tests] [bench-args...]
TAG=${1:-q}
FOCUS=${2:--}
MODE=${3:-tests}
shift 3 2>/dev/null
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
if [ "$FOCUS" != "-" ]; then
  timeout -k 10 400 python3 -u -m pytest $FOCUS -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_focus.log 2>&1 || { tail -30 gpurun_out/${TAG}_focus.log; exit 1; }
  tail -2 gpurun_out/${TAG}_focus.log
fi
if [ "$MODE" = tests ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
  tail -2 gpurun_out/${TAG}_gputest.log
fi
timeout -k 10 300 python3 bench.py --steps 256 --skip-cpu --seq-reps 2 --batch "" --abi-steps 32 "$@" > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
grep -E "decode:|seq-eval|ABI|k_qgemm|seq GEMM" gpurun_out/${TAG}_bench.log
if [ -f rwkv.cppy_amd/build_stamp/librwkv.so ]; then
  timeout -k 10 200 python3 tools/stamp_run.py v6-1b6-q4_0 > gpurun_out/${TAG}_stamps.txt 2>&1 || { tail -5 gpurun_out/${TAG}_stamps.txt; exit 1; }
  sed -n 1,10p gpurun_out/${TAG}_stamps.txt
fi

# A/B (optional): AB="ENV=VAL" runs the decode-only bench once more with that environment
if [ -n "$AB" ]; then
  env $AB timeout -k 10 200 python3 bench.py --decode-only --steps 256 > gpurun_out/${TAG}_ab.log 2>&1 || { tail -5 gpurun_out/${TAG}_ab.log; exit 1; }
  echo "A/B $AB:"; grep -E "decode:" gpurun_out/${TAG}_ab.log
  timeout -k 10 200 python3 bench.py --decode-only --steps 256 > gpurun_out/${TAG}_ab0.log 2>&1 || { tail -5 gpurun_out/${TAG}_ab0.log; exit 1; }
  echo "A/B default:"; grep -E "decode:" gpurun_out/${TAG}_ab0.log
fi
echo done
