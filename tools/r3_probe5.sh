#!/bin/bash
# ABI host-state decode under copy-engine runtime settings (pageable and page-locked buffers)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in X=0 DEBUG_CLR_LIMIT_BLIT_WG=16 DEBUG_CLR_LIMIT_BLIT_WG=64 GPU_BLIT_ENGINE_TYPE=1 GPU_BLIT_ENGINE_TYPE=2 "RWKV_MI355X_IO_PIPELINE=0 DEBUG_CLR_LIMIT_BLIT_WG=16"; do
  env $v timeout -k 10 200 python3 bench.py --steps 16 --skip-cpu --seq-reps 0 --batch "" --abi-steps 64 --timing-steps 1 > gpurun_out/p5_ab.log 2>&1 || { tail -5 gpurun_out/p5_ab.log; exit 1; }
  grep -E "ABI" gpurun_out/p5_ab.log | sed "s/^/[$v] /"
done
echo done
