#!/bin/bash
# PMC passes (SQ counters) over the _1-format m*s pass (k_qg_msum*) of a v5-7B sequence
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
n=0
for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"; do
  n=$((n+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-trace --kernel-include-regex "k_qg_msum" -d $ROOT/gpurun_out/pms_$n -o run --output-format csv -- \
      python3 $ROOT/bench.py --config v5-7b-q4_1 --steps 2 --warmup 1 --skip-cpu --seq-reps 1 --abi-steps 0 --timing-steps 1 --batch "" --pipe-stages 0 \
      > $ROOT/gpurun_out/pms_$n.log 2>&1 || exit $?
done
cd $ROOT && python3 tools/pmc_agg.py gpurun_out/pms_1 "1>" ; python3 tools/pmc_agg.py gpurun_out/pms_2 "1>"
