#!/bin/bash
# sequence-eval A/B over environment knobs: tools/r5_abseq.sh CONFIG "ENV1" ...  ("-" = defaults)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=$GRAFT_REPO_ROOT/gpurun_out
c=$1; shift
for e in "$@"; do
  [ "$e" = "-" ] && e=""
  env $e timeout -k 10 300 python3 bench.py --config $c --steps 4 --warmup 1 --batch "" --seq-reps 5 --abi-steps 0 --skip-cpu --pipe-stages 0 \
    > $O/abs.json 2> $O/abs.err || { tail -5 $O/abs.err; exit 1; }
  echo "$c [$e] $(grep -E 'seq-eval T|self-check' $O/abs.err | tr '\n' ' ')"
done
