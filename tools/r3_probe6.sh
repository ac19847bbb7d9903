#!/bin/bash
# Decode phase stamps with the chain's shader clock (stamp build), then the ABI copy-engine A/B.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 200 python3 tools/stamp_run.py v6-1b6-q4_0 > gpurun_out/p6_stamps.txt 2>&1 || { tail -5 gpurun_out/p6_stamps.txt; exit 1; }
head -20 gpurun_out/p6_stamps.txt
bash tools/r3_probe5.sh
