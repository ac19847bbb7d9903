#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/r8_tests.log 2>&1
rc=$?; tail -2 $O/r8_tests.log; grep FAILED $O/r8_tests.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
tools/r5_ab.sh v5-7b-q4_1 - RWKV_MI355X_LN_R8=0 && tools/r5_ab.sh v7-2b9-q5_1 - RWKV_MI355X_LN_R8=0
