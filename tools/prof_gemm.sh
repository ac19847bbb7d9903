#!/bin/bash
# PMC passes over tools/gemm_probe variants (qgemm only).  Usage: tools/prof_gemm.sh TAG
TAG=${1:-x}
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in "" _p1 _p2; do
  n=0
  for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
    n=$((n+1))
    timeout -k 10 120 rocprofv3 --pmc $ctr --kernel-trace -d $ROOT/gpurun_out/pg_${TAG}${v}_$n -o run --output-format csv -- $ROOT/tools/gemm_probe$v 1 > $ROOT/gpurun_out/pg_${TAG}${v}_$n.log 2>&1 || exit $?
  done
done
