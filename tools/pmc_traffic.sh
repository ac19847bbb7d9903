#!/bin/bash
# HBM traffic of the decode kernels from PMC counters (MI355X_MICROARCH.md, HBM section):
# separate passes for FETCH_SIZE and WRITE_SIZE (they do not fit one pass), kernel trace only,
# no runtime/sys tracing.  Output: gpurun_out/pmc_<TAG>_{fetch,write}/ then tools/pmc_summary.py.
TAG=${1:-x}
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $ROOT/gpurun_out/pmc_${TAG}_fetch -o run \
    --output-format csv -- python3 $ROOT/bench.py --steps 32 --warmup 8 --skip-cpu --seq-reps 0 --abi-steps 0 --batch "" \
    > $ROOT/gpurun_out/pmc_${TAG}_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $ROOT/gpurun_out/pmc_${TAG}_write -o run \
    --output-format csv -- python3 $ROOT/bench.py --steps 32 --warmup 8 --skip-cpu --seq-reps 0 --abi-steps 0 --batch "" \
    > $ROOT/gpurun_out/pmc_${TAG}_write.log 2>&1
