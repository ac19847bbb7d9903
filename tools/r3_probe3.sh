#!/bin/bash
# GEMM epilogue A/B (packed vs scalar f32; tools/gemm_probe variants, outputs hashed) and a HIP API
# trace of the page-locked ABI decode.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in gemm_probe gemm_probe_s gemm_probe_s2 gemm_probe; do
  echo "== $v"; timeout -k 10 120 tools/pbin/$v 1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace -d $GRAFT_REPO_ROOT/gpurun_out/abihip -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --skip-cpu --seq-reps 0 --batch "" --abi-steps 16 --timing-steps 1 \
  > $GRAFT_REPO_ROOT/gpurun_out/abihip.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/abihip.log; exit 1; }
grep ABI $GRAFT_REPO_ROOT/gpurun_out/abihip.log
echo done
