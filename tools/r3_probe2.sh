#!/bin/bash
# New replica / state-slice GPU tests, then an A/B of the ABI host-state decode (chunk sizes,
# whole-state path) with pageable and page-locked buffers.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_replicas.py tests/test_gpu_pipeline.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/p2_tests.log 2>&1 || { tail -40 gpurun_out/p2_tests.log; exit 1; }
tail -3 gpurun_out/p2_tests.log
for v in RWKV_MI355X_IO_CHUNK=4 RWKV_MI355X_IO_CHUNK=2 RWKV_MI355X_IO_CHUNK=6 RWKV_MI355X_IO_CHUNK=12 RWKV_MI355X_IO_PIPELINE=0; do
  env $v timeout -k 10 200 python3 bench.py --steps 16 --skip-cpu --seq-reps 0 --batch "" --abi-steps 64 --timing-steps 1 > gpurun_out/p2_ab.log 2>&1 || { tail -5 gpurun_out/p2_ab.log; exit 1; }
  grep -E "ABI" gpurun_out/p2_ab.log | sed "s/^/[$v] /"
done
echo done
