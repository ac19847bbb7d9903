#!/bin/bash
# full GPU suite after the _1 split / fmm split.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/p24_gputest.log 2>&1 || { tail -30 gpurun_out/p24_gputest.log; exit 1; }
tail -1 gpurun_out/p24_gputest.log
