#!/bin/bash
# decode A/B over environment knobs: tools/r5_ab.sh CONFIG "ENV1" "ENV2" ...  ("-" = defaults)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=$GRAFT_REPO_ROOT/gpurun_out
c=$1; shift
for e in "$@"; do
  [ "$e" = "-" ] && e=""
  env $e timeout -k 10 200 python3 bench.py --config $c --decode-only --steps 128 --warmup 16 --skip-cpu --pipe-stages 0 \
    > $O/ab.json 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
  echo "$c [$e] $(grep 'decode:' $O/ab.err)"
done
