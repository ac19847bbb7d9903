#!/bin/bash
# Sequence-path A/B (round 4): the bench's seq-eval + GEMM lines for build_alt/librwkv.so and for
# the product build, same box, back to back.  Usage: tools/r4_ab_seq.sh TAG [config]
TAG=${1:-ab}
CFG=${2:-v6-1b6-q4_0}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for arm in alt prod alt2 prod2; do
  case $arm in alt*) LIBV=rwkv.cppy_amd/build_alt/librwkv.so ;; *) LIBV= ;; esac
  RWKV_MI355X_BENCH_LIB=$LIBV timeout -k 10 300 python3 bench.py --config $CFG --steps 16 --skip-cpu --seq-reps 3 --batch "" --abi-steps 0 > gpurun_out/${TAG}_${arm}.log 2>&1 || { tail -5 gpurun_out/${TAG}_${arm}.log; exit 1; }
  echo "== $arm"; grep -E "seq-eval|k_qgemm|seq GEMM" gpurun_out/${TAG}_${arm}.log
done
