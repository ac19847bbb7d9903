#!/bin/bash
# Interleaved A/B of builds of the library on one box: bench.py --decode-only (graph-replayed
# device-resident decode), alternating between arms.  An arm is LABEL=LIB[@ENV=VALUE...]: LIB
# "this" is this tree's build, anything else a path handed to bench.py as RWKV_MI355X_BENCH_LIB;
# the optional ENV assignments are exported for that arm only.
# Usage: tools/ab_lib.sh CONFIG REPS ARM [ARM ...]
#   tools/ab_lib.sh v6-1b6-q4_0 3 r5=rwkv.cppy_amd/build_r5/librwkv.so head=this head-noffn=this@RWKV_MI355X_DECODE_FUSION=191
CFG=$1
REPS=$2
shift 2
for i in $(seq $REPS); do
  for arm in "$@"; do
    label=${arm%%=*}
    rest=${arm#*=}
    lib=${rest%%@*}
    envs=""
    [ "$rest" != "$lib" ] && envs=${rest#*@}
    (
      if [ "$lib" = this ]; then unset RWKV_MI355X_BENCH_LIB; else export RWKV_MI355X_BENCH_LIB=$lib; fi
      for e in ${envs//@/ }; do export "$e"; done
      timeout -k 10 200 python bench.py --config $CFG --decode-only --steps 256 --warmup 32 --skip-cpu 2>&1 >/dev/null \
        | grep "decode:" | sed "s/^/[$label] /"
    ) || exit 1
  done
done
