#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 300 python -u -m pytest "tests/test_gpu_configs.py::test_config_decode_bit_exact" "tests/test_gpu_batch.py::test_batch_real_width_bit_exact" -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread > $O/u8.log 2>&1
rc=$?; echo "rc=$rc $(tail -1 $O/u8.log)"; grep FAILED $O/u8.log
if [ $rc -ne 0 ]; then exit $rc; fi
tools/r5_ab.sh v7-2b9-q5_1 - RWKV_MI355X_ACT_U8=0 - RWKV_MI355X_ACT_U8=0
