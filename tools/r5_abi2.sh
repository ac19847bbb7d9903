#!/bin/bash
# ABI decode: rate A/B of the copy-stream queue knobs, then a kernel + memory-copy trace of one knob
cd $GRAFT_REPO_ROOT
tools/r5_abiab.sh "X=0" "RWKV_MI355X_IO_PRIO=1" "RWKV_MI355X_IO_PRIO=1 RWKV_MI355X_IO_CHUNK=2" "RWKV_MI355X_IO_PRIO=1 RWKV_MI355X_IO_CHUNK=3" || exit 1
export RWKV_MI355X_IO_PRIO=1
cd /tmp && export TMPDIR=/tmp
for k in pageable pinned; do
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $GRAFT_REPO_ROOT/gpurun_out/abip_$k -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/tools/abi_trace.py $k 24 > $GRAFT_REPO_ROOT/gpurun_out/abip_$k.log 2>&1 || exit 1
done
