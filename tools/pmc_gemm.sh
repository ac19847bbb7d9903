#!/bin/bash
# PMC passes over the sequence GEMM (k_qgemm*) in a short bench run, one counter group per pass
# (rocprofv3 does not split passes), kernel trace only.  Usage: tools/pmc_gemm.sh TAG
TAG=${1:-x}
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
n=0
for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -d $ROOT/gpurun_out/pmcg_${TAG}_$n -o run --output-format csv -- \
      python3 $ROOT/bench.py --steps 2 --warmup 1 --skip-cpu --seq-reps 1 --abi-steps 0 --timing-steps 1 --batch "" \
      > $ROOT/gpurun_out/pmcg_${TAG}_$n.log 2>&1 || exit $?
done
