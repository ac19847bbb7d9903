#!/bin/bash
# Round-3 probe 1: decode front-end counters (tools/r3_icache.sh) and a kernel + memory-copy trace
# of the ABI decode with pageable and page-locked host state.  Stops at the first failure.
ROOT=$GRAFT_REPO_ROOT
cd $ROOT && mkdir -p gpurun_out
bash tools/r3_icache.sh ic > gpurun_out/ic.log 2>&1 || { tail -20 gpurun_out/ic.log; exit 1; }
cat gpurun_out/ic.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d $ROOT/gpurun_out/abitrace -o run --output-format csv -- \
  python3 $ROOT/bench.py --steps 2 --warmup 1 --skip-cpu --seq-reps 0 --batch "" --abi-steps 8 --timing-steps 1 \
  > $ROOT/gpurun_out/abitrace.log 2>&1 || { tail -5 $ROOT/gpurun_out/abitrace.log; exit 1; }
echo done
