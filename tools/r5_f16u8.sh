#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/f16_tests.log 2>&1
rc=$?; tail -2 $O/f16_tests.log; grep FAILED $O/f16_tests.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
tools/r5_ab.sh v7-2b9-q5_1 - RWKV_MI355X_F16_U8=0 - RWKV_MI355X_F16_U8=0
