#!/bin/bash
# packed-vs-scalar f32 probe and the host cost of the decode graph launch
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 60 tools/pbin/pk_probe || exit 1
timeout -k 10 200 python3 tools/host_probe.py v6-1b6-q4_0 300 || exit 1
timeout -k 10 200 python3 tools/host_probe.py v4-169m-q8_0 300 || exit 1
echo done
