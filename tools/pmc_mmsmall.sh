#!/bin/bash
# SQ counters of k_mm_small / k_wkv7_s64 in the v7 sequence workload (tools/, on the GPU box).
# One --pmc pass with --kernel-trace --stats only, bounded by its own time limit.
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --kernel-include-regex 'k_mm_small|k_wkv7_s64' \
  --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU \
  -d $ROOT/gpurun_out/pmc_mms -o run --output-format csv -- \
  python3 $ROOT/bench.py --config v7-2b9-q5_1 --steps 2 --warmup 1 --skip-cpu --seq-reps 1 --abi-steps 0 --batch "" \
  --timing-steps 1 > $ROOT/gpurun_out/pmc_mms.log 2>&1
