#!/bin/bash
# PMC passes (SQ counters) over the sequence GEMM of a library variant: tools/r5_pmcq.sh TAG LIBDIR QG32
ROOT=$GRAFT_REPO_ROOT
TAG=$1
export RWKV_MI355X_BENCH_LIB=$ROOT/rwkv.cppy_amd/$2/librwkv.so RWKV_MI355X_QG32=$3
cd /tmp && export TMPDIR=/tmp
n=0
for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --kernel-include-regex "k_qg" -d $ROOT/gpurun_out/pq_${TAG}_$n -o run --output-format csv -- \
      python3 $ROOT/bench.py --steps 2 --warmup 1 --skip-cpu --seq-reps 1 --abi-steps 0 --timing-steps 1 --batch "" --pipe-stages 0 \
      > $ROOT/gpurun_out/pq_${TAG}_$n.log 2>&1 || exit $?
done
cd $ROOT && python3 tools/pmc_agg.py gpurun_out/pq_${TAG}_1 "1>" ; python3 tools/pmc_agg.py gpurun_out/pq_${TAG}_2 "1>"
