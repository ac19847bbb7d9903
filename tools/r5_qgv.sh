#!/bin/bash
# (GPU box) sequence + batched timing of library variants built by tools/qgvar.sh, k_qg32 on.
# Usage: tools/r5_qgv.sh NAME... (env CFG = bench config, BATCH = batched sizes, QG32 = 0/1)
cd ${GRAFT_REPO_ROOT:-/root/repo}
for n in "$@"; do
  RWKV_MI355X_QG32=${QG32:-1} RWKV_MI355X_BENCH_LIB=$PWD/rwkv.cppy_amd/build_$n/librwkv.so BATCH=${BATCH:-} \
    CFG=${CFG:-v6-1b6-q4_0} tools/ab_seq.sh "VARIANT=$n" | grep -v '^.*{"metric'
done
