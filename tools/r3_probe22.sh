#!/bin/bash
# NaN hunt in the float matmul (fmm) path.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 120 python3 -u tools/fmm_nan_probe.py 2>&1 | tee gpurun_out/p22.txt
