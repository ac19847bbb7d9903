#!/bin/bash
# bit-exactness of a knob (v7 / v5 config tests) then decode A/B
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=$GRAFT_REPO_ROOT/gpurun_out
KNOB=$1
env $KNOB timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > $O/ab2_tests.log 2>&1
rc=$?; tail -2 $O/ab2_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for c in v7-2b9-q5_1 v5-7b-q4_1; do
  for e in - "$KNOB" - "$KNOB"; do
    [ "$e" = "-" ] && e=""
    env $e timeout -k 10 200 python3 bench.py --config $c --decode-only --steps 128 --warmup 16 --skip-cpu --pipe-stages 0 \
      > $O/ab.json 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
    echo "$c [$e] $(grep 'decode:' $O/ab.err)"
  done
done
