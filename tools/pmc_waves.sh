#!/bin/bash
# Wave-lifetime counters of the decode kernels (one --pmc pass, kernel trace only).
TAG=${1:-x}
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $ROOT/gpurun_out/pmcw_${TAG} -o run \
    --output-format csv -- python3 $ROOT/bench.py --steps 8 --warmup 4 --skip-cpu --seq-reps 0 --abi-steps 0 \
    > $ROOT/gpurun_out/pmcw_${TAG}.log 2>&1
