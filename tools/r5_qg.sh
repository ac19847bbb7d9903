#!/bin/bash
# k_qg32 (RWKV_MI355X_QG32=1): GEMM / sequence / batched parity tests, then sequence and batched A/B.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${1:-q}
RWKV_MI355X_QG32=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py \
  tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -15 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
BATCH=128 tools/ab_seq.sh RWKV_MI355X_QG32=0 RWKV_MI355X_QG32=1
CFG=v7-2b9-q5_1 tools/ab_seq.sh RWKV_MI355X_QG32=0 RWKV_MI355X_QG32=1
