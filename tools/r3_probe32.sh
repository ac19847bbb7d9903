#!/bin/bash
# fmm K/T/M sweep (per-workgroup fixed cost) + the round-3c cycle (GPU tests, smoke, bench, rocprof).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 120 tools/pbin/fmm_probe > gpurun_out/p32_fmm.txt 2>&1 || { cat gpurun_out/p32_fmm.txt; exit 1; }
cat gpurun_out/p32_fmm.txt
bash tools/r3_cycle.sh r3c tests || exit 1
grep -E "decode|seq-eval" gpurun_out/r3c_bench.log | cut -c1-160
echo done
