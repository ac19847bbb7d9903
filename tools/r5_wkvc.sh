#!/bin/bash
# chunk-parallel wkv6: tests, kernel timings (rocprofv3), seq-eval A/B through bench.py
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_wkv_chunk.py -x -q -s -p no:cacheprovider --timeout 300 \
  --timeout-method thread > $O/wkvc_tests.log 2>&1
rc=$?
grep -E "relative|dlogit|passed|failed|Error|assert" $O/wkvc_tests.log | head -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc $rc"; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/wkvc_prof -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/tools/wkv_chunk_time.py > $O/wkvc_prof.log 2>&1 || { tail -5 $O/wkvc_prof.log; exit 1; }
grep "relative" $O/wkvc_prof.log
grep -E "wkv" $(find $O/wkvc_prof -name "*kernel_stats.csv") | cut -c1-150
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 bench.py --steps 16 --warmup 4 --batch "" --abi-steps 0 --skip-cpu --pipe-stages 0 --seq-reps 3 \
  > $O/wkvc_bench.json 2> $O/wkvc_bench.err || { tail -5 $O/wkvc_bench.err; exit 1; }
grep -E "seq-eval" $O/wkvc_bench.err
