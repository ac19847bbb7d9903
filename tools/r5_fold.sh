#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/fold_tests.log 2>&1
rc=$?; tail -2 $O/fold_tests.log; grep FAILED $O/fold_tests.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
for c in v6-1b6-q4_0 v7-2b9-q5_1 v5-7b-q4_1; do
  timeout -k 10 300 python3 bench.py --config $c --steps 8 --warmup 2 --batch "128" --seq-reps 3 --abi-steps 0 --skip-cpu --pipe-stages 0 > $O/fo.json 2> $O/fo.err || { tail -5 $O/fo.err; exit 1; }
  echo "$c $(grep -E 'seq-eval T|batched decode B=128|self-check|seq GEMM' $O/fo.err | tr '\n' ' ')"
done
