#!/bin/bash
# ABI decode traces (tools/abi_trace.py) for pageable and page-locked caller buffers:
# rate first, then rocprofv3 --kernel-trace --memory-copy-trace (no PMC), CSV under gpurun_out/.
ROOT=$GRAFT_REPO_ROOT
TAG=${1:-abi}
cd $ROOT
for k in pageable pinned; do
  timeout -k 10 120 python3 tools/abi_trace.py $k 64 || exit 1
done
cd /tmp && export TMPDIR=/tmp
for k in pageable pinned; do
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $ROOT/gpurun_out/${TAG}_$k -o run --output-format csv -- \
    python3 $ROOT/tools/abi_trace.py $k 24 > $ROOT/gpurun_out/${TAG}_$k.log 2>&1 || { tail -5 $ROOT/gpurun_out/${TAG}_$k.log; exit 1; }
done
cd $ROOT && python3 tools/abi_timeline.py gpurun_out/${TAG}_pageable gpurun_out/${TAG}_pinned
